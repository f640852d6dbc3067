cd "${GRAFT_REPO_ROOT:-/root/repo}"
REPO=$(pwd)
mkdir -p gpurun_out/r5
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sweeps.py tests/test_gpu_fe.py tests/test_gpu_amg.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r5/tests_sub.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 gpurun_out/r5/tests_sub.log; [ $rc -eq 0 ] || exit $rc
dir=$REPO/gpurun_out/r5/fe12_fact; rm -rf $dir; mkdir -p $dir
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$dir" -o run -- python3 "$REPO/bench.py" --system fe --N 12 --inner ilu --steps 1 --warmup 0 --maxit 5 --no-cpu --no-copy-probe > "$dir/stdout.log" 2>&1) || exit 1
rm -f $dir/run_kernel_trace.csv
python3 -c "
import csv
rows=list(csv.DictReader(open('$dir/run_kernel_stats.csv')))
for r in rows[:6]: print(r['Name'][:60], r['Calls'], 'total ms', round(float(r['TotalDurationNs'])/1e6,1), 'avg us', round(float(r['AverageNs'])/1e3,1))"
grep setup $dir/stdout.log | head -3
bash tools/r5_c21.sh
