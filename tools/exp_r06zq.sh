#!/bin/bash
# The fused edge evaluation in the batched pose kernel: pose GPU tests, then the bench's pose legs (1024-frame batches)
# against the previous commit (posehead), twice.
set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_pose_gpu.py tests/test_pose_lastframe_gpu.py tests/test_pose_edges_gpu.py > gpurun_out/r06zq_tests.log 2>&1 || { tail -30 gpurun_out/r06zq_tests.log; exit 1; }
tail -2 gpurun_out/r06zq_tests.log
ARGS="--steps 2 --warmup 1 --no-cpu-baseline --stage-timing 0 --parity-check 0 --lba-steps 0 --tri-pairs 0 --aux 0 --p1080-frames 0 --latency-frames 0"
for i in 1 2; do
  for v in product posehead; do
    if [ $v == product ]; then L=""; else L=openmavis_amd/variants/libomv_$v.so; fi
    OMV_LIB=$L timeout -k 10 300 python3 tools/bench_lib.py $ARGS 2> gpurun_out/r06zq_$v.err | tail -1 | python3 -c "
import json,sys
d=json.loads(sys.stdin.read())
print('$v', {k: d[k]['value'] for k in ('pose_inertial','pose_inertial_last_frame','pose_optimization','pose_optimization_b1') if k in d})" >> gpurun_out/r06zq_ab.log || exit 1
  done
  tail -5 gpurun_out/r06zq_product.err
done
cat gpurun_out/r06zq_ab.log
