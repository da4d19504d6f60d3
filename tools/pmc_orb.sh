#!/bin/bash
# One PMC pass (<= 8 SQ counters) over tools/orb_once.py; per-kernel sums per wave.
# bash tools/pmc_orb.sh <tag> "<counters>"   (on the box, from the repo root)
set -euo pipefail
TAG=${1:-orbpmc}
CTR=${2:-"SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS"}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc $CTR -d $OUT/orb -o run --output-format csv -- python3 $R/tools/orb_once.py --frames 32 --reps 1 > /dev/null 2>&1
python3 - $OUT <<'PY'
import csv, sys, collections, re, os
d = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(os.path.join(sys.argv[1], "orb", "run_counter_collection.csv"))):
    m = re.search(r"::(\w+_kernel)", r["Kernel_Name"])
    if m:
        d[m.group(1)][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in d.items():
    w = max(v.get("SQ_WAVES", 1), 1)
    print(k, " ".join(f"{c}={v[c]/w:.1f}/wave" if c != "SQ_WAVES" else f"waves={v[c]:.0f}" for c in sorted(v)))
PY
