cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5
timeout -k 10 900 python -u -m pytest tests/test_dist_gpu.py -k "g4_g8" -v --timeout 850 --timeout-method thread -p no:cacheprovider > gpurun_out/r5/dist_big.log 2>&1; rc=$?
echo "dist big rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/r5/dist_big.log | tail -12
exit $rc
