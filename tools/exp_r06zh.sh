#!/bin/bash
# Same-box A/B of the LocalBA solver: the product against the library before the substitution split (lbaold):
# optimize() wall times (median of 20, alternating, three times), the rocprof timeline and per-level profiles.
set -uo pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
for i in 1 2 3; do
  for v in product lbaold; do
    if [ $v == product ]; then L=""; else L=openmavis_amd/variants/libomv_$v.so; fi
    OMV_LIB=$L timeout -k 10 120 python3 tools/lba_time.py 20 > gpurun_out/r06zh_$v.jsonl 2>&1 || exit 1
    python3 -c "
import json,sys,statistics as st
rs=[json.loads(l) for l in open('gpurun_out/r06zh_$v.jsonl') if l.startswith('{')]
print('$v', 'median wall_ms %.4f' % st.median(r['wall_ms'] for r in rs[2:]), {k: round(st.median(r[k] for r in rs[2:]),4) for k in rs[0] if k not in ('wall_ms','err','err_end')})
" >> gpurun_out/r06zh_ab.log
  done
done
bash tools/ldlt_ab.sh lbaold -- ldltprof lbaoldprof >> gpurun_out/r06zh_ab.log 2>&1
cat gpurun_out/r06zh_ab.log | head -60
