set -e
mkdir -p gpurun_out
for i in 1 2; do
for v in pyr8 pyr32; do
OMV_LIB=openmavis_amd/variants/libomv_$v.so timeout -k 10 120 python3 tools/orb_once.py --frames 128 --reps 5 --timing 2>&1 | grep images | sed "s/^/$v /" >> gpurun_out/r06x_ab.log
done
timeout -k 10 120 python3 tools/orb_once.py --frames 128 --reps 5 --timing 2>&1 | grep images | sed "s/^/pyr16 /" >> gpurun_out/r06x_ab.log
done
