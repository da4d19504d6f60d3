#!/bin/bash
# LocalInertialBA per-kernel timeline of one optimize() (rocprofv3 kernel trace of tools/lba_time.py).
set -euo pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace -d $R/gpurun_out/lbatl -o run --output-format csv -- python3 $R/tools/lba_time.py 3 > /dev/null 2>&1
python3 $R/tools/lba_timeline.py $R/gpurun_out/lbatl/run_kernel_trace.csv | tail -60
