cd "${GRAFT_REPO_ROOT:-/root/repo}"
REPO=$(pwd)
mkdir -p gpurun_out/r5
timeout -k 10 400 python -u -m pytest tests/test_gpu_sweeps.py -v -k swin --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r5/sweeps_test.log 2>&1 ; rc=$?; echo "swin tests rc=$rc"; [ $rc -eq 0 ] || exit $rc
profrun() {  # profrun <dir> <bench args...>
    local dir=$REPO/gpurun_out/r5/$1; shift
    rm -rf "$dir"; mkdir -p "$dir"
    (cd /tmp && export TMPDIR=/tmp && timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$dir" -o run -- python3 "$REPO/bench.py" "$@" > "$dir/stdout.log" 2>&1)
    local rc=$?
    rm -f "$dir"/run_kernel_trace.csv
    echo "== $1 rc=$rc $(grep '^{' $dir/stdout.log | cut -c90-135)"
    python3 -c "
import csv
rows=list(csv.DictReader(open('$dir/run_kernel_stats.csv')))
for r in rows[:3]: print(r['Name'][:40], r['Calls'], 'avg us', round(float(r['AverageNs'])/1e3,1))"
    return $rc
}
profrun fe12_swin --system fe --N 12 --inner ilu --steps 2 --warmup 1 --no-cpu --no-copy-probe --opt pls.sweep_swin=1
