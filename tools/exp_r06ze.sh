#!/bin/bash
# Forward / backward substitution over lane groups: LDL^T timeline + per-level profile, LBA tests (product and the
# all-global variant).
set -uo pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
bash $R/tools/ldlt_ab.sh gcur -- ldltprof > $R/gpurun_out/r06ze_ab.log 2>&1 || exit 1
cd $R && timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_lba_gpu.py > gpurun_out/r06ze_lba_tests.log 2>&1 || exit 1
tail -2 gpurun_out/r06ze_lba_tests.log
OMV_LIB=openmavis_amd/variants/libomv_gcur.so timeout -k 10 300 python -u tools/pytest_lib.py -x -q --timeout 200 --timeout-method thread tests/test_lba_gpu.py > gpurun_out/r06ze_lba_tests_gcur.log 2>&1
tail -2 gpurun_out/r06ze_lba_tests_gcur.log
