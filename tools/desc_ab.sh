set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_orb_gpu.py > gpurun_out/r06e_tests.log 2>&1
for i in 1 2; do
for v in pw1 pw2 pw8; do
echo "== $v" >> gpurun_out/r06e_ab.log
OMV_LIB=openmavis_amd/variants/libomv_$v.so timeout -k 10 120 python3 tools/orb_once.py --frames 128 --reps 5 --timing >> gpurun_out/r06e_ab.log 2>&1
done
echo "== pw4" >> gpurun_out/r06e_ab.log
timeout -k 10 120 python3 tools/orb_once.py --frames 128 --reps 5 --timing >> gpurun_out/r06e_ab.log 2>&1
done
