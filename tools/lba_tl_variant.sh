#!/bin/bash
# LocalInertialBA kernel timeline of one optimize() with an instrumented library variant:
# bash tools/lba_tl_variant.sh <variant name>   (openmavis_amd/variants/libomv_<name>.so)
set -euo pipefail
R=$GRAFT_REPO_ROOT
V=$1
cd /tmp && export TMPDIR=/tmp
export OMV_LIB=$R/openmavis_amd/variants/libomv_$V.so
timeout -k 10 120 rocprofv3 --kernel-trace -d $R/gpurun_out/lbatl_$V -o run --output-format csv -- python3 $R/tools/lba_time.py 3 > /dev/null 2>&1
python3 $R/tools/lba_timeline.py $R/gpurun_out/lbatl_$V/run_kernel_trace.csv | head -40
