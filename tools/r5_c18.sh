cd "${GRAFT_REPO_ROOT:-/root/repo}"
REPO=$(pwd)
mkdir -p gpurun_out/r5
profrun() {  # profrun <dir> <bench args...>
    local dir=$REPO/gpurun_out/r5/$1; shift
    rm -rf "$dir"; mkdir -p "$dir"
    (cd /tmp && export TMPDIR=/tmp && timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$dir" -o run -- python3 "$REPO/bench.py" "$@" > "$dir/stdout.log" 2>&1)
    local rc=$?
    rm -f "$dir"/run_kernel_trace.csv
    python3 -c "
import csv
rows=list(csv.DictReader(open('$dir/run_kernel_stats.csv')))
for r in rows[:1]: print('$dir'.split('/')[-1], r['Name'][:40], r['Calls'], 'avg us', round(float(r['AverageNs'])/1e3,1))"
    return $rc
}
for p in 0 512 1024; do
profrun fe12_swin_p$p --system fe --N 12 --inner ilu --steps 1 --warmup 0 --maxit 20 --no-cpu --no-copy-probe --opt pls.sweep_swin=1 --opt pls.ring_probe=$p || exit 1
done
