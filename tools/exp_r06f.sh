set -e
mkdir -p gpurun_out
for i in 1 2; do
echo "== default" >> gpurun_out/r06f_pyr.log
timeout -k 10 120 python3 tools/orb_once.py --frames 128 --reps 5 --timing >> gpurun_out/r06f_pyr.log 2>&1
echo "== chain" >> gpurun_out/r06f_pyr.log
OMV_PYR_MODE=chain timeout -k 10 120 python3 tools/orb_once.py --frames 128 --reps 5 --timing >> gpurun_out/r06f_pyr.log 2>&1
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_lba_gpu.py > gpurun_out/r06f_lba_tests.log 2>&1
OMV_LIB=openmavis_amd/variants/libomv_skippad.so timeout -k 10 300 python -u tools/pytest_lib.py -x -q --timeout 200 --timeout-method thread tests/test_lba_gpu.py > gpurun_out/r06f_lba_tests_skippad.log 2>&1 || true
bash tools/ldlt_ab.sh skippad > gpurun_out/r06f_ldlt_ab.log 2>&1
