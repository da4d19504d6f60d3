#!/bin/bash
# Phase profile of the B=1 pose kernels after the private-stack fix, with the LastFrame EdgeInertial wave split into
# error / Jacobian / info*J.
set -uo pipefail
mkdir -p gpurun_out
OMV_LIB=openmavis_amd/variants/libomv_poseprof.so timeout -k 10 120 python3 tools/pose_latency.py --pts 4300 --stereo 0.36 --modes grouped --parts 0 --reps 1 > gpurun_out/r06zj_poseprof.log 2>&1
grep -v "^$" gpurun_out/r06zj_poseprof.log | grep -v amdgpu.ids | head -40
