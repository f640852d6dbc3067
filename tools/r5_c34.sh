# headline setup with the one-launch factorization against per-level launches
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5
for dep in 2 0; do
  timeout -k 10 400 python3 bench.py --steps 3 --warmup 1 --no-cpu --no-copy-probe --opt pls.ilu_factor_dep=$dep > gpurun_out/r5/c34_dep$dep.log 2>&1 || { tail -20 gpurun_out/r5/c34_dep$dep.log; exit 1; }
  echo "dep=$dep: $(grep -E '^\[bench\] setup' gpurun_out/r5/c34_dep$dep.log) $(tail -1 gpurun_out/r5/c34_dep$dep.log | cut -c1-120)"
done
