#!/bin/bash
# LDL^T plan A/B: blocks in global scratch with the two-chain order (gcur) and with recursive dissection (gnd),
# against the product (LDS, two chains); per-level profiles; the LBA tests on the dissection variant.
set -uo pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
bash $R/tools/ldlt_ab.sh gcur gnd gndg -- ldltprof gndprof > $R/gpurun_out/r06zd_ab.log 2>&1 || exit 1
cd $R && OMV_LIB=openmavis_amd/variants/libomv_gnd.so timeout -k 10 300 python -u tools/pytest_lib.py -x -q --timeout 200 --timeout-method thread tests/test_lba_gpu.py > gpurun_out/r06zd_lba_tests_gnd.log 2>&1
tail -3 gpurun_out/r06zd_lba_tests_gnd.log
