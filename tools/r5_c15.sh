cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5
timeout -k 10 400 python -u -m pytest tests/test_gpu_sweeps.py -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r5/sweeps_test.log 2>&1 ; rc=$?; echo "sweeps rc=$rc"; grep -E "PASSED|FAILED|Error|error" gpurun_out/r5/sweeps_test.log | head -20; exit $rc
