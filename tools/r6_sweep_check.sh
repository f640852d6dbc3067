#!/bin/bash
# round 6: the tests touching the window sweeps, then the level-0 sweep per launch at swelling N=80 / 160
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out/r6
timeout -k 10 700 python -u -m pytest tests/test_gpu_sweeps.py tests/test_gpu_harness.py tests/test_gpu_amg.py tests/test_gpu_fe.py \
    tests/test_gpu_cg_device.py -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r6/win_tests2.log 2>&1
rc=$?; grep -E "passed|failed" gpurun_out/r6/win_tests2.log | tail -n 2; grep FAILED gpurun_out/r6/win_tests2.log | head -3; [ $rc -eq 0 ] || exit $rc
bash tools/r6_sweep_ab.sh h80 swelling 80 || exit $?
bash tools/r6_sweep_ab.sh h160 swelling 160 || exit $?
