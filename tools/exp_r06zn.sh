#!/bin/bash
# LDL^T: each inverse wave reads its next level's task before the barrier.  LBA GPU tests, then same-box A/B of
# optimize() against the previous commit (lbaold), the rocprof timeline and the per-level profile.
set -uo pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_lba_gpu.py > gpurun_out/r06zn_tests.log 2>&1 || { tail -30 gpurun_out/r06zn_tests.log; exit 1; }
tail -2 gpurun_out/r06zn_tests.log
for i in 1 2 3; do
  for v in product lbaold; do
    if [ $v == product ]; then L=""; else L=openmavis_amd/variants/libomv_$v.so; fi
    OMV_LIB=$L timeout -k 10 120 python3 tools/lba_time.py 20 > gpurun_out/r06zn_$v.jsonl 2>&1 || exit 1
    python3 -c "
import json,statistics as st
rs=[json.loads(l) for l in open('gpurun_out/r06zn_$v.jsonl') if l.startswith('{')]
print('lba $v median wall_ms %.4f' % st.median(r['wall_ms'] for r in rs[2:]))" >> gpurun_out/r06zn_ab.log
  done
done
bash tools/ldlt_ab.sh lbaold -- ldltprof >> gpurun_out/r06zn_ab.log 2>&1
head -40 gpurun_out/r06zn_ab.log
