set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_orb_gpu.py tests/test_bench_shape_gpu.py tests/test_p1080_gpu.py > gpurun_out/r06u_tests.log 2>&1
for i in 1 2 3; do
timeout -k 10 120 python3 tools/orb_once.py --frames 128 --reps 5 --timing 2>&1 | grep images >> gpurun_out/r06u_ab.log
done
