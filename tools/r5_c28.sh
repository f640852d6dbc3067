cd "${GRAFT_REPO_ROOT:-/root/repo}"
REPO=$(pwd)
mkdir -p gpurun_out/r5
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sweeps.py tests/test_gpu_fe.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r5/tests_sub2.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 gpurun_out/r5/tests_sub2.log; [ $rc -eq 0 ] || exit $rc
dir=$REPO/gpurun_out/r5/fe12_fact; rm -rf $dir; mkdir -p $dir
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$dir" -o run -- python3 "$REPO/bench.py" --system fe --N 12 --inner ilu --steps 1 --warmup 0 --maxit 5 --no-cpu --no-copy-probe > "$dir/stdout.log" 2>&1) || exit 1
rm -f $dir/run_kernel_trace.csv
python3 -c "
import csv
rows=list(csv.DictReader(open('$dir/run_kernel_stats.csv')))
for r in rows[:3]: print(r['Name'][:60], r['Calls'], 'total ms', round(float(r['TotalDurationNs'])/1e6,1), 'avg us', round(float(r['AverageNs'])/1e3,1))"
grep "setup" $dir/stdout.log | head -2
for rep in 1; do
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu --no-copy-probe > gpurun_out/r5/head_$rep.log 2>&1 || exit 1
echo "head $rep $(grep '^{' gpurun_out/r5/head_$rep.log | cut -c90-130)"
done
