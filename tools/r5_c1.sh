cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5
timeout -k 10 300 python -u -m pytest tests/test_gpu_sweeps.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r5/sweeps_test.log 2>&1 ; echo "sweeps rc=$?"
tail -3 gpurun_out/r5/sweeps_test.log
timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu --no-copy-probe --opt pls.sweep_profile=1 --opt pls.ilu_view=1 > gpurun_out/r5/prof_blocks.log 2>&1 && echo prof ok &&
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu --no-copy-probe --opt pls.sweep_tpb=256 > gpurun_out/r5/tpb256.log 2>&1 && echo tpb ok &&
grep '^{' gpurun_out/r5/tpb256.log | cut -c1-300
