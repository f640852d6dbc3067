#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out/r6
timeout -k 10 400 python -u -m pytest tests/test_gpu_sweeps.py tests/test_gpu_fe.py tests/test_gpu_harness.py -m gpu -x -v --timeout 120 --timeout-method thread \
    -p no:cacheprovider -k "window or harness" > gpurun_out/r6/win16_tests.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error|passed|failed" gpurun_out/r6/win16_tests.log | tail -n 20; [ $rc -eq 0 ] || exit $rc
bash tools/r6_sweep_ab.sh f80 swelling 80 || exit $?
bash tools/r6_sweep_ab.sh f160 swelling 160 || exit $?
