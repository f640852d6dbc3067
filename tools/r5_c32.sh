# per-row phase times of the ILU(0) factorization (pls.ilu0_probe), FE 3-D N=12
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5
for dep in 1 0; do
  timeout -k 10 300 python3 bench.py --system fe --N 12 --inner ilu --steps 1 --warmup 0 --maxit 2 --no-cpu --no-copy-probe --opt pls.ilu_factor_dep=$dep --opt pls.ilu0_probe=97 > gpurun_out/r5/c32_dep$dep.log 2>&1 || { tail -20 gpurun_out/r5/c32_dep$dep.log; exit 1; }
  grep -c "ilu0 row" gpurun_out/r5/c32_dep$dep.log
done
