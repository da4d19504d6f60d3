set -e
mkdir -p gpurun_out
timeout -k 10 60 ./tools/micro/ldlt24_v2 > gpurun_out/r06m_ldlt_v3.log 2>&1
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_orb_gpu.py tests/test_bench_shape_gpu.py > gpurun_out/r06m_tests.log 2>&1
for i in 1 2; do
timeout -k 10 120 python3 tools/orb_once.py --frames 128 --reps 5 --timing >> gpurun_out/r06m_ab.log 2>&1
done
