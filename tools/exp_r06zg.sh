#!/bin/bash
# describe with K output slots per wave (orientations of K keypoints at once, patches re-staged): ORB GPU tests on
# the product (K = 4), then isolated extraction timings of K = 1 / 2 / 4 / 8, twice.
set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_orb_gpu.py > gpurun_out/r06zg_tests.log 2>&1 || { tail -30 gpurun_out/r06zg_tests.log; exit 1; }
tail -2 gpurun_out/r06zg_tests.log
for i in 1 2; do
for v in 1 2 8 4w8; do
OMV_LIB=openmavis_amd/variants/libomv_desck$v.so timeout -k 10 120 python3 tools/orb_once.py --frames 128 --reps 5 --timing 2>&1 | grep images | sed "s/^/K=$v /" >> gpurun_out/r06zg_ab.log || exit 1
done
timeout -k 10 120 python3 tools/orb_once.py --frames 128 --reps 5 --timing 2>&1 | grep images | sed "s/^/K=4 /" >> gpurun_out/r06zg_ab.log || exit 1
done
cat gpurun_out/r06zg_ab.log
