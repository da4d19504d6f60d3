#!/bin/bash
# SearchByProjection candidate stage on the GPU box: matcher parity tests, then per-stage times of one 128-frame
# stream group for the global-memory kernel and the LDS-staged one at several chunk sizes (OMV_CAND_PW).
set -euo pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 240 python -u -m pytest tests/test_match_gpu.py tests/test_p1080_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/cs_tests.log 2>&1 || { tail -30 gpurun_out/cs_tests.log; exit 1; }
tail -1 gpurun_out/cs_tests.log
echo "== global"
OMV_CAND=global timeout -k 10 120 python tools/match_once.py --frames 128 --reps 3 --timing 2>&1 | grep frames
for PW in "$@"; do
  echo "== lds pw $PW"
  OMV_CAND_PW=$PW timeout -k 10 120 python tools/match_once.py --frames 128 --reps 3 --timing 2>&1 | grep frames
done
