#!/bin/bash
# Quick LocalInertialBA iteration on the GPU box: the LBA GPU tests, one optimize() timeline, the LBA bench leg and
# the FETCH_SIZE / WRITE_SIZE passes of tools/lba_time.py (summarised with tools/summarize_profile.py <tag>).
# Usage (on the box, from the repo root): bash tools/quick_lba.sh <tag>
set -euo pipefail
TAG=${1:-qlba}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_lba_gpu.py \
    > gpurun_out/ql_tests.log 2>&1 || { tail -30 gpurun_out/ql_tests.log; exit 1; }
tail -1 gpurun_out/ql_tests.log
bash tools/lba_tl.sh
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 1 --warmup 1 --pose-frames 0 --tri-pairs 0 --aux 0 \
    --p1080-frames 0 --latency-frames 0 > gpurun_out/ql_bench.json 2> gpurun_out/ql_bench.err
python3 -c "
import json; d = json.loads(open('gpurun_out/ql_bench.json').read().strip().splitlines()[-1]); l = d['local_ba']
print('LBA', l['value'], l['ms_per_trial'], l['ms_per_optimize'], l['stage_ms_per_trial'], l['err_end'])"
cd /tmp && export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C -T -d $OUT/pmc_lba_$C -o run --output-format csv -- \
      python3 $R/tools/lba_time.py 2 > $OUT/lba_$C.txt 2> $OUT/lba_$C.err
done
echo done
