set -e
mkdir -p gpurun_out
OMV_FAST_LDS_PRINT=1 timeout -k 10 120 python3 tools/orb_once.py --frames 128 --reps 5 --timing 2>&1 | grep -E 'images|LDS' >> gpurun_out/r06zb_ab.log
for pad in 0 1024 2048 0 1024 2048; do
OMV_FAST_LDS_PAD=$pad timeout -k 10 120 python3 tools/orb_once.py --frames 128 --reps 5 --timing 2>&1 | grep images | sed "s/^/pad=$pad /" >> gpurun_out/r06zb_ab.log
done
