set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_pose_gpu.py tests/test_pose_lastframe_gpu.py tests/test_pose_edges_gpu.py tests/test_cpp_consumer_gpu.py > gpurun_out/r06n_tests.log 2>&1
timeout -k 10 120 python3 tools/pose_latency.py --pts 4300 --stereo 0.36 --modes grouped --parts 0 --reps 20 > gpurun_out/r06n_pose.log 2>&1
OMV_LIB=openmavis_amd/variants/libomv_poseprof.so timeout -k 10 120 python3 tools/pose_latency.py --pts 4300 --stereo 0.36 --modes grouped --parts 0 --reps 1 > gpurun_out/r06n_poseprof.log 2>&1
