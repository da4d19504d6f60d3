#!/bin/bash
# Final check at HEAD: the whole GPU suite and smoke().
set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/r06zr_gputests.log 2>&1 || { tail -30 gpurun_out/r06zr_gputests.log; exit 1; }
tail -2 gpurun_out/r06zr_gputests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" 2>&1 | tail -2
