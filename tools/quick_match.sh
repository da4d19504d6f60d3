#!/bin/bash
# Quick matcher iteration on the GPU box: matcher parity tests, isolated stage times of one 128-frame group
# (tools/match_once.py --timing) and the HBM fetch of its kernels (one FETCH_SIZE pass on 32 frames).
set -euo pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 200 python -u -m pytest tests/test_match_gpu.py tests/test_p1080_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/qm_tests.log 2>&1 || { tail -30 gpurun_out/qm_tests.log; exit 1; }
tail -1 gpurun_out/qm_tests.log
timeout -k 10 120 python tools/match_once.py --frames 128 --reps 3 --timing
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/qm_pmc -o run --output-format csv -- python3 $R/tools/match_once.py --frames 32 --reps 1 > /dev/null 2>&1
python3 - $R/gpurun_out/qm_pmc/run_counter_collection.csv <<'PY'
import csv, sys, collections, re
d = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    m = re.search(r"::(\w+_kernel)", r["Kernel_Name"])
    d[m.group(1) if m else r["Kernel_Name"][:40]].append(float(r["Counter_Value"]))
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1]))[:10]:
    print(f"{k:40s} FETCH_SIZE {sum(v)/len(v)/1024:9.1f} MB/launch (x2 gfx950: {2*sum(v)/len(v)/1024:9.1f})")
PY
