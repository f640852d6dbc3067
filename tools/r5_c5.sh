cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5
for v in "-1 -1" "2 -1" "-1 0" "2 0"; do
set -- $v
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu --no-copy-probe --opt pls.ilu_view=1 --opt pls.fp_pipeline_rr=$1 --opt pls.fp_pipeline_lds=$2 > gpurun_out/r5/pipe_$1_$2.log 2>&1 || exit 1
echo "rr=$1 lds=$2 $(grep -o 'round-robin groups.*' gpurun_out/r5/pipe_$1_$2.log) $(grep '^{' gpurun_out/r5/pipe_$1_$2.log | cut -c90-130)"
done
bash tools/r5_trace.sh on
