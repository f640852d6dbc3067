cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5
timeout -k 10 300 python -u bench.py --steps 1 --warmup 0 --no-cpu --no-copy-probe --opt pls.ilu_view=2 > gpurun_out/r5/ilu_view2.log 2>&1 && echo ok
grep "pls ilu" gpurun_out/r5/ilu_view2.log
