#!/bin/bash
# GPU call (tag as $1, default r03i): BoW / SearchForInitialization parity + timing first, then the full round (tests, bench, profile, smoke).
# Continues past a test failure (rc 1) only; any other status (timeout, fault, abort) ends the call.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_bowmatch_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/bowinit.log 2>&1
rc=$?; tail -3 gpurun_out/bowinit.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 200 python -u tools/bow_once.py > gpurun_out/bow_once.txt 2>&1 || exit $?
tail -4 gpurun_out/bow_once.txt
bash tools/gpu_round.sh ${1:-r03i} || exit $?
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')"
