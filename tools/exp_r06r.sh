set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_lba_gpu.py > gpurun_out/r06r_tests.log 2>&1
bash tools/lba_tl.sh > gpurun_out/r06r_lbatl.log 2>&1
timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 --lba-steps 30 > gpurun_out/r06r_bench.json 2> gpurun_out/r06r_bench.err
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_orb_gpu.py tests/test_bench_shape_gpu.py tests/test_p1080_gpu.py > gpurun_out/r06r_orbtests.log 2>&1
for i in 1 2; do
timeout -k 10 120 python3 tools/orb_once.py --frames 128 --reps 5 --timing >> gpurun_out/r06r_ab.log 2>&1
done
