cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5
for d in 6 2; do for l in -1 0; do
timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-cpu --no-copy-probe --opt pls.ilu_view=3 --opt pls.fp_pipeline_depth=$d --opt pls.fp_pipeline_lds=$l > gpurun_out/r5/pipe_prof_d${d}_l$l.log 2>&1 || exit 1
echo "depth=$d lds=$l"; grep "fp pipeline\]" gpurun_out/r5/pipe_prof_d${d}_l$l.log | grep -v first
done; done
