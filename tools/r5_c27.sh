cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5
for rep in 1 2; do
for v in "pls.fp_pipeline=0" "pls.fp_pipeline_cus=0" "pls.fp_pipeline=1"; do
  timeout -k 10 300 python -u bench.py --inner hypre --steps 3 --warmup 1 --no-cpu --no-copy-probe --opt $v --opt pls.spmv_short=0 > gpurun_out/r5/abh2_$v.log 2>&1 || exit 1
  echo "hypre $rep $v $(grep '^{' gpurun_out/r5/abh2_$v.log | cut -c90-130)"
done; done
