#!/bin/bash
# Octree kernel A/B on the GPU box: ORB parity tests, then per-stage times of one stream group at B=1 and B=128.
set -euo pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_orb_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/oct_tests.log 2>&1 || { tail -30 gpurun_out/oct_tests.log; exit 1; }
tail -1 gpurun_out/oct_tests.log
for B in 1 2 128; do
  timeout -k 10 120 python tools/match_once.py --frames $B --reps 5 --timing 2>&1 | grep frames
done
