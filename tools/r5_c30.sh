# one-launch ILU(0) factorization: bitwise test, FE / parity ILU tests, then
# the FE N=12 and N=24 factorization kernels' durations (rocprofv3 kernel trace)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
REPO=$(pwd)
mkdir -p gpurun_out/r5
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_fe.py -k "factor_dep or gmem_sweep" > gpurun_out/r5/c30_tests.log 2>&1 || { tail -30 gpurun_out/r5/c30_tests.log; exit 1; }
tail -5 gpurun_out/r5/c30_tests.log
for N in 12 24; do
  dir=$REPO/gpurun_out/r5/fe${N}_dep; rm -rf $dir; mkdir -p $dir
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$dir" -o run -- python3 "$REPO/bench.py" --system fe --N $N --inner ilu --steps 1 --warmup 0 --maxit 2 --no-cpu --no-copy-probe > "$dir/stdout.log" 2>&1) || { tail -20 $dir/stdout.log; exit 1; }
  f=$(find $dir -name '*kernel_stats.csv' | head -1)
  grep -E "Name|k_ilu0|k_ilu_blocks" $f | cut -c1-200
  find $dir -name '*kernel_trace.csv' -delete
done
