cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5
timeout -k 10 300 python -u -m pytest tests/test_gpu_sweeps.py -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r5/sweeps_test.log 2>&1 ; rc=$?; echo "sweeps rc=$rc"; tail -3 gpurun_out/r5/sweeps_test.log; [ $rc -eq 0 ] || exit $rc
for d in 6 2; do
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu --no-copy-probe --opt pls.ilu_view=1 --opt pls.fp_pipeline_depth=$d > gpurun_out/r5/pipe_d$d.log 2>&1 || exit 1
echo "depth=$d $(grep -o 'sweep tpb.*' gpurun_out/r5/pipe_d$d.log) $(grep '^{' gpurun_out/r5/pipe_d$d.log | cut -c90-130)"
done
bash tools/r5_trace.sh on
