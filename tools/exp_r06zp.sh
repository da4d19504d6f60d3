#!/bin/bash
# the visual edge's projection and Jacobian side by side: pose GPU tests, then B=1 latency against the
# previous commit (posehead), then the phase profile.
set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_pose_gpu.py tests/test_pose_lastframe_gpu.py tests/test_pose_edges_gpu.py tests/test_cpp_consumer_gpu.py > gpurun_out/r06zp_tests.log 2>&1 || { tail -30 gpurun_out/r06zp_tests.log; exit 1; }
tail -2 gpurun_out/r06zp_tests.log
for i in 1 2; do
  for v in product posehead; do
    if [ $v == product ]; then L=""; else L=openmavis_amd/variants/libomv_$v.so; fi
    OMV_LIB=$L timeout -k 10 120 python3 tools/pose_latency.py --pts 4300 --stereo 0.36 --modes grouped --parts 0 --reps 30 2>/dev/null | grep '^{' | sed "s/^/$v /" >> gpurun_out/r06zp_ab.log || exit 1
  done
done
cat gpurun_out/r06zp_ab.log
OMV_LIB=openmavis_amd/variants/libomv_poseprof.so timeout -k 10 120 python3 tools/pose_latency.py --pts 4300 --stereo 0.36 --modes grouped --parts 0 --reps 1 2>&1 | grep "pose_lat<1>" | head -8
