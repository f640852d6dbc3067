# one-launch ILU(0) factorization (relaxed polls) against the per-level launches
cd "${GRAFT_REPO_ROOT:-/root/repo}"
REPO=$(pwd)
mkdir -p gpurun_out/r5
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_fe.py -k "factor_dep" > gpurun_out/r5/c31_tests.log 2>&1 || { tail -30 gpurun_out/r5/c31_tests.log; exit 1; }
tail -3 gpurun_out/r5/c31_tests.log
for N in 12 24; do
 for dep in 1 0; do
  dir=$REPO/gpurun_out/r5/fe${N}_dep$dep; rm -rf $dir; mkdir -p $dir
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$dir" -o run -- python3 "$REPO/bench.py" --system fe --N $N --inner ilu --steps 1 --warmup 0 --maxit 2 --no-cpu --no-copy-probe --opt pls.ilu_factor_dep=$dep > "$dir/stdout.log" 2>&1) || { tail -20 $dir/stdout.log; exit 1; }
  f=$(find $dir -name '*kernel_stats.csv' | head -1)
  echo "N=$N dep=$dep"; grep -E "k_ilu0" $f | cut -c1-30,120-220
  find $dir -name '*kernel_trace.csv' -delete
 done
done
