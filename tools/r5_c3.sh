cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5
timeout -k 10 300 python -u -m pytest tests/test_gpu_sweeps.py -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r5/sweeps_test.log 2>&1 ; rc=$?; echo "sweeps rc=$rc"; tail -5 gpurun_out/r5/sweeps_test.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu --no-copy-probe --opt pls.ilu_view=1 > gpurun_out/r5/pipe_on.log 2>&1 && echo on ok && grep "fp pipeline\|^{" gpurun_out/r5/pipe_on.log | cut -c1-400 &&
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu --no-copy-probe --opt pls.fp_pipeline=0 > gpurun_out/r5/pipe_off.log 2>&1 && echo off ok && grep "^{" gpurun_out/r5/pipe_off.log | cut -c1-300
