cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5
timeout -k 10 300 python -u -m pytest tests/test_gpu_sweeps.py -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r5/sweeps_test.log 2>&1 ; rc=$?; echo "sweeps rc=$rc"; tail -2 gpurun_out/r5/sweeps_test.log; [ $rc -eq 0 ] || exit $rc
for v in "-1 2" "-1 6" "0 2"; do set -- $v
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu --no-copy-probe --opt pls.ilu_view=3 --opt pls.fp_pipeline_cus=$1 --opt pls.fp_pipeline_depth=$2 > gpurun_out/r5/pipe_cus$1_d$2.log 2>&1 || exit 1
echo "cus=$1 depth=$2 $(grep '^{' gpurun_out/r5/pipe_cus$1_d$2.log | cut -c90-130)"; grep "fp pipeline\]" gpurun_out/r5/pipe_cus$1_d$2.log | cut -c1-250
done
bash tools/r5_trace.sh on
