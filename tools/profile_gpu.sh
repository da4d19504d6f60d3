#!/bin/bash
# Round profile on the GPU box: kernel-trace stats of the default bench, then separate PMC passes
# (FETCH_SIZE, WRITE_SIZE) on the extraction/matching kernels.  Output under gpurun_out/prof_<tag>/.
# Usage (on the box, from the repo root): bash tools/profile_gpu.sh <tag> [bench args...]
set -euo pipefail
TAG=${1:-r01}; shift || true
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $OUT/trace -o run --output-format csv -- \
    python3 $R/bench.py --no-cpu-baseline "$@" > $OUT/bench_trace.json 2> $OUT/bench_trace.err
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C -T -d $OUT/pmc_$C -o run --output-format csv -- \
      python3 $R/bench.py --no-cpu-baseline --stage-timing 0 "$@" > $OUT/bench_$C.json 2> $OUT/bench_$C.err
done
echo done
