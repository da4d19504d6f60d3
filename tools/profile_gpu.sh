#!/bin/bash
# Round profile on the GPU box: kernel-trace stats of the default bench (short), then separate PMC passes
# (FETCH_SIZE, WRITE_SIZE) on one batched ORB extraction of 32 frames x 5 cameras, twice (tools/orb_once.py:
# 160 images per launch).  Output under gpurun_out/prof_<tag>/.
# Usage (on the box, from the repo root): bash tools/profile_gpu.sh <tag>
set -euo pipefail
TAG=${1:-r01}; shift || true
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
# heartbeat under gpurun_out/ (the traced bench prints only at its end); each step keeps its own timeout
( while sleep 20; do date >> $OUT/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T -d $OUT/trace -o run --output-format csv -- \
    python3 $R/bench.py --no-cpu-baseline --steps 5 --warmup 1 --lba-steps 3 --pose-frames 256 --tri-pairs 64 \
    > $OUT/bench_trace.json 2> $OUT/bench_trace.err
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C -T -d $OUT/pmc_$C -o run --output-format csv -- \
      python3 $R/tools/orb_once.py --frames 32 --reps 2 > $OUT/orb_$C.txt 2> $OUT/orb_$C.err
done
echo done
