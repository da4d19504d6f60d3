#!/bin/bash
# Instruction mix / stall split of the ORB and matcher kernels (one --pmc pass each program, 8 SQ counters):
# bash tools/pmc_mix.sh <tag>   (on the box, from the repo root)
set -euo pipefail
TAG=${1:-mix}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
CTR="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
timeout -s KILL 120 rocprofv3 --pmc $CTR -d $OUT/orb -o run --output-format csv -- python3 $R/tools/orb_once.py --frames 32 --reps 1 > /dev/null 2>&1
timeout -s KILL 120 rocprofv3 --pmc $CTR -d $OUT/match -o run --output-format csv -- python3 $R/tools/match_once.py --frames 32 --reps 1 > /dev/null 2>&1
python3 - $OUT <<'PY'
import csv, sys, collections, re, os
for prog in ("orb", "match"):
    d = collections.defaultdict(lambda: collections.defaultdict(float))
    n = collections.Counter()
    for r in csv.DictReader(open(os.path.join(sys.argv[1], prog, "run_counter_collection.csv"))):
        m = re.search(r"::(\w+_kernel)", r["Kernel_Name"])
        if not m:
            continue
        d[m.group(1)][r["Counter_Name"]] += float(r["Counter_Value"])
    print(f"== {prog}")
    for k, v in sorted(d.items(), key=lambda kv: -kv[1]["SQ_WAVE_CYCLES"]):
        w = max(v["SQ_WAVES"], 1)
        print(f"{k:22s} waves {v['SQ_WAVES']:9.0f} cyc/wave {4*v['SQ_WAVE_CYCLES']/w:8.0f} active {v['SQ_ACTIVE_INST_ANY']/max(v['SQ_WAVE_CYCLES'],1):5.2f} "
              f"wait {v['SQ_WAIT_ANY']/max(v['SQ_WAVE_CYCLES'],1):5.2f} waitinst {v['SQ_WAIT_INST_ANY']/max(v['SQ_WAVE_CYCLES'],1):5.2f} "
              f"valu/wave {v['SQ_INSTS_VALU']/w:8.0f} lds/wave {v['SQ_INSTS_LDS']/w:7.0f} busy {v['SQ_BUSY_CYCLES']:10.0f}")
PY
