#!/bin/bash
# PoseOptimization (pose_only_kernel) with the fused mono projection + Jacobian: its GPU tests, then B=1 / B=256
# timings against the previous commit (posehead).
set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_pose_only_gpu.py tests/test_cpp_consumer_gpu.py > gpurun_out/r06zs_tests.log 2>&1 || { tail -30 gpurun_out/r06zs_tests.log; exit 1; }
tail -2 gpurun_out/r06zs_tests.log
for i in 1 2; do
  for v in product posehead; do
    if [ $v == product ]; then L=""; else L=openmavis_amd/variants/libomv_$v.so; fi
    for F in 1 256; do
      OMV_LIB=$L timeout -k 10 120 python3 tools/po_time.py $F 30 2>/dev/null | grep -v amdgpu.ids | tail -1 | sed "s/^/$v F=$F /" >> gpurun_out/r06zs_ab.log || exit 1
    done
  done
done
cat gpurun_out/r06zs_ab.log
