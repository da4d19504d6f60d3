#!/bin/bash
# One GPU call: GPU tests, the default bench, then the rocprof kernel-trace + PMC profile.
# Usage (on the box, from the repo root): bash tools/gpu_round.sh <tag> [skip-tests]
set -euo pipefail
TAG=${1:-r02}
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
if [ "${2:-}" != "skip-tests" ]; then
  timeout -k 10 400 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread \
      > gpurun_out/gputests_$TAG.log 2>&1
  tail -3 gpurun_out/gputests_$TAG.log
fi
timeout -k 10 500 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
tail -c 600 gpurun_out/bench_$TAG.json
bash tools/profile_gpu.sh $TAG
bash tools/pmc_orb_bound.sh bound_$TAG
