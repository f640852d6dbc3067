cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5
for lay in 1 0; do
bash tools/r5_trace.sh lay$lay --opt pls.fp_pipeline_cu_layout=$lay | head -9
done
for v in "1 -1" "1 8" "1 24" "0 8"; do set -- $v
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu --no-copy-probe --opt pls.fp_pipeline_cu_layout=$1 --opt pls.fp_pipeline_cus=$2 > gpurun_out/r5/pipe_lay$1_cus$2.log 2>&1 || exit 1
echo "layout=$1 cus=$2 $(grep '^{' gpurun_out/r5/pipe_lay$1_cus$2.log | cut -c90-130)"
done
