cd "${GRAFT_REPO_ROOT:-/root/repo}"
REPO=$(pwd)
mkdir -p gpurun_out/r5
profrun() {  # profrun <dir> <bench args...>
    local dir=$REPO/gpurun_out/r5/$1; shift
    rm -rf "$dir"; mkdir -p "$dir"
    (cd /tmp && export TMPDIR=/tmp && timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$dir" -o run -- python3 "$REPO/bench.py" "$@" > "$dir/stdout.log" 2>&1)
    local rc=$?
    rm -f "$dir"/run_kernel_trace.csv
    echo "== $dir rc=$rc $(grep '^{' $dir/stdout.log | cut -c90-135)"
    head -4 $dir/run_kernel_stats.csv | cut -c1-60,200-320
    return $rc
}
profrun fe12_swin --system fe --N 12 --inner ilu --steps 2 --warmup 1 --no-cpu --no-copy-probe --opt pls.sweep_swin=1 || exit 1
profrun fe12_ring --system fe --N 12 --inner ilu --steps 2 --warmup 1 --no-cpu --no-copy-probe --opt pls.sweep_swin=0 || exit 1
profrun fe24_swin --system fe --N 24 --inner ilu --steps 1 --warmup 1 --maxit 10 --no-cpu --no-copy-probe --opt pls.sweep_swin=1 || exit 1
