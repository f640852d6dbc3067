cd "${GRAFT_REPO_ROOT:-/root/repo}"
REPO=$(pwd)
dir=$REPO/gpurun_out/r5/fe12_ftrace; rm -rf $dir; mkdir -p $dir
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$dir" -o run -- python3 "$REPO/bench.py" --system fe --N 12 --inner ilu --steps 1 --warmup 0 --maxit 2 --no-cpu --no-copy-probe > "$dir/stdout.log" 2>&1) || exit 1
f=$(find $dir -name '*kernel_trace.csv' | head -1)
head -1 $f | cut -c1-400
python3 tools/trace_kernel_hist.py $f k_ilu0_level
rm -f $f
