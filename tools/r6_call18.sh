#!/bin/bash
# round 6: ring / mixed window sweeps -- tests, then N=160 kernel stats (default = mixed, and both-windows)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out/r6
timeout -k 10 300 python -u -m pytest tests/test_gpu_sweeps.py -m gpu -x -v --timeout 120 --timeout-method thread \
    -p no:cacheprovider -k "window" > gpurun_out/r6/ring_tests.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error|passed|failed" gpurun_out/r6/ring_tests.log | tail -n 12; [ $rc -eq 0 ] || exit $rc
bash tools/r6_call17.sh
