set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_lba_gpu.py tests/test_pose_gpu.py tests/test_pose_lastframe_gpu.py tests/test_pose_edges_gpu.py tests/test_cpp_consumer_gpu.py > gpurun_out/r06zc_tests.log 2>&1
timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 --lba-steps 30 > gpurun_out/r06zc_bench.json 2> gpurun_out/r06zc_bench.err
