#!/bin/bash
# Round profile on the GPU box: kernel-trace stats of the default bench (short), then separate PMC passes
# (FETCH_SIZE, WRITE_SIZE) on three short programs with homogeneous launches:
#   orb   tools/orb_once.py   --frames 32 --reps 2   (one extraction launch = 160 images)
#   match tools/match_once.py --frames 32 --reps 2   (one stream group of the headline pipeline, 32 frames)
#   lba   tools/lba_time.py 2                        (LocalInertialBA optimize() on the configs[4] window)
# Output under gpurun_out/prof_<tag>/.  Usage (on the box, from the repo root): bash tools/profile_gpu.sh <tag>
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
  timeout -k 10 300 rocprofv3 --pmc $C -T -d $OUT/pmc_orb_$C -o run --output-format csv -- \
      python3 $R/tools/orb_once.py --frames 32 --reps 2 > $OUT/orb_$C.txt 2> $OUT/orb_$C.err
  timeout -k 10 300 rocprofv3 --pmc $C -T -d $OUT/pmc_match_$C -o run --output-format csv -- \
      python3 $R/tools/match_once.py --frames 32 --reps 2 > $OUT/match_$C.txt 2> $OUT/match_$C.err
  timeout -k 10 300 rocprofv3 --pmc $C -T -d $OUT/pmc_lba_$C -o run --output-format csv -- \
      python3 $R/tools/lba_time.py 2 > $OUT/lba_$C.txt 2> $OUT/lba_$C.err
done
echo done
