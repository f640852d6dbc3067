cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5
for v in "none" "pls.fp_pipeline=0" "pls.spmv_short=0" "pls.hypre_coarsen_chunks=0"; do
  o=""; [ "$v" != none ] && o="--opt $v"
  timeout -k 10 300 python -u bench.py --inner hypre --steps 3 --warmup 1 --no-cpu --no-copy-probe $o > gpurun_out/r5/hyp59_$v.log 2>&1 || exit 1
  echo "$v: $(grep -o 'setup [0-9.]* s' gpurun_out/r5/hyp59_$v.log | head -1) $(grep -o 'warmup solve: [0-9]* its' gpurun_out/r5/hyp59_$v.log) $(grep '^{' gpurun_out/r5/hyp59_$v.log | cut -c90-130)"
done
