#!/bin/bash
# SearchByProjection candidate / resolve A/B on the GPU box: parity tests of the matcher, per-stage times of one
# stream group at B=1 and B=128 for the candidate kernels (OMV_CAND=global vs LDS-staged), and the resolve walk's
# per-domain blocks / rounds from instrumented builds (variants/libomv_<name>.so given as arguments).
set -euo pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 240 python -u -m pytest tests/test_match_gpu.py tests/test_p1080_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/rab_tests.log 2>&1 || { tail -30 gpurun_out/rab_tests.log; exit 1; }
tail -1 gpurun_out/rab_tests.log
for B in 1 128; do
  echo "== B=$B LDS-staged candidates"
  timeout -k 10 120 python tools/match_once.py --frames $B --reps 3 --timing
  echo "== B=$B global candidates"
  OMV_CAND=global timeout -k 10 120 python tools/match_once.py --frames $B --reps 3 --timing
done
for V in "$@"; do
  echo "== resolve profile $V (B=2)"
  OMV_LIB=openmavis_amd/variants/libomv_$V.so timeout -k 10 120 python tools/match_once.py --frames 2 --reps 1 2>&1 | grep resolve || true
done
