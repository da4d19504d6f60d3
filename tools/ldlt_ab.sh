#!/bin/bash
# LDL^T A/B on the GPU box: the LocalInertialBA timeline (ldlt / err rows) of the product library and of the
# variants named on the command line, then the per-level phase printout of the OMV_LDLT_PROFILE variants.
# Usage (on the box, from the repo root): bash tools/ldlt_ab.sh <variant>... [-- <profile variant>...]
set -uo pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
run_tl() {
  local lib=$1 tag=$2
  OMV_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace -d $R/gpurun_out/ab_$tag -o run --output-format csv -- \
      python3 $R/tools/lba_time.py 3 > /dev/null 2>&1 || { echo "$tag: failed"; return 1; }
  echo "== $tag"; python3 $R/tools/lba_timeline.py $R/gpurun_out/ab_$tag/run_kernel_trace.csv | tail -8
}
run_tl $R/openmavis_amd/libomv_hip.so product || exit 1
prof=0
for v in "$@"; do
  if [ "$v" == "--" ]; then prof=1; continue; fi
  if [ $prof == 0 ]; then run_tl $R/openmavis_amd/variants/libomv_$v.so $v || exit 1
  else
    echo "== profile $v"
    OMV_LIB=$R/openmavis_amd/variants/libomv_$v.so timeout -k 10 120 python3 $R/tools/lba_time.py 1 2>&1 | grep -E "ldlt|level" | head -24 || exit 1
  fi
done
