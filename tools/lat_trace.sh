#!/bin/bash
# Kernel-trace the B=1 latency leg (rocprofv3 --kernel-trace --stats) and print the per-kernel averages.
# Usage (on the box, from the repo root): bash tools/lat_trace.sh <tag>
set -euo pipefail
TAG=${1:-lat}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- \
    python3 $R/bench.py --frames 3 --streams 1 --steps 1 --warmup 1 --latency-frames 200 --no-cpu-baseline \
    --lba-steps 0 --pose-frames 0 --tri-pairs 0 --aux 0 --p1080-frames 0 --stage-timing 0 > $OUT/bench.json 2> $OUT/bench.err
python3 - $OUT/run_kernel_stats.csv <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = 0.0
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:22]:
    print(f"{r['Name'][:58]:58s} {r['Calls']:>6} avg {float(r['AverageNs'])/1e3:8.1f} us  min {float(r['MinNs'])/1e3:8.1f}")
PY
tail -c 300 $OUT/bench.json
