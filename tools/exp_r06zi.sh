#!/bin/bash
# Private-stack fixes: LDL^T block locator as a value type (no scratch), the pose edge Jacobian with constant trip
# counts (pr / JP in registers).  LBA + pose GPU tests, then same-box A/B: LocalBA optimize() against lbaold, the
# B=1 pose latency against poseold.
set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_lba_gpu.py tests/test_pose_gpu.py tests/test_pose_lastframe_gpu.py tests/test_pose_edges_gpu.py tests/test_pose_only_gpu.py > gpurun_out/r06zi_tests.log 2>&1 || { tail -30 gpurun_out/r06zi_tests.log; exit 1; }
tail -2 gpurun_out/r06zi_tests.log
for i in 1 2; do
  for v in product lbaold; do
    if [ $v == product ]; then L=""; else L=openmavis_amd/variants/libomv_$v.so; fi
    OMV_LIB=$L timeout -k 10 120 python3 tools/lba_time.py 20 > gpurun_out/r06zi_$v.jsonl 2>&1 || exit 1
    python3 -c "
import json,statistics as st
rs=[json.loads(l) for l in open('gpurun_out/r06zi_$v.jsonl') if l.startswith('{')]
print('lba $v median wall_ms %.4f' % st.median(r['wall_ms'] for r in rs[2:]))" >> gpurun_out/r06zi_ab.log
  done
  for v in product poseold; do
    if [ $v == product ]; then L=""; else L=openmavis_amd/variants/libomv_$v.so; fi
    OMV_LIB=$L timeout -k 10 120 python3 tools/pose_latency.py --pts 4300 --stereo 0.36 --modes grouped --parts 0 --reps 30 2>/dev/null | grep '^{' | sed "s/^/$v /" >> gpurun_out/r06zi_ab.log || exit 1
  done
done
cat gpurun_out/r06zi_ab.log
