set -e
mkdir -p gpurun_out
OMV_LIB=openmavis_amd/variants/libomv_poseprof.so timeout -k 10 120 python3 tools/pose_latency.py --pts 4300 --stereo 0.36 --modes grouped --parts 0 --reps 1 > gpurun_out/r06za_poseprof.log 2>&1
