#!/bin/bash
# Quick extractor iteration on the GPU box: ORB parity tests (incl. 1080p and the bench's own shape), isolated
# per-stage times of one 128-frame launch set (tools/orb_once.py --timing) and a short headline bench.
set -euo pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 400 python -u -m pytest tests/test_orb_gpu.py tests/test_p1080_gpu.py tests/test_bench_shape_gpu.py -x -q \
    --timeout 480 --timeout-method thread > gpurun_out/qo_tests.log 2>&1 || { tail -30 gpurun_out/qo_tests.log; exit 1; }
tail -1 gpurun_out/qo_tests.log
timeout -k 10 120 python tools/orb_once.py --frames 128 --reps 3 --timing
timeout -k 10 300 python bench.py --no-cpu-baseline --lba-steps 0 --pose-frames 0 --tri-pairs 0 --aux 0 \
    --p1080-frames 0 --latency-frames 0 > gpurun_out/qo_bench.json 2> gpurun_out/qo_bench.err
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/qo_bench.json").read().strip().splitlines()[-1])
print("value", d["value"], "ms/step", d["ms_per_step"], "parity", d.get("parity_post_run", {}).get("bit_exact"))
print("stage ms/step", d.get("stage_ms_per_step"))
print({k: v.get("isolated", {}).get("avg_launch_ms") for k, v in d.get("kernels", {}).items()})
PY
