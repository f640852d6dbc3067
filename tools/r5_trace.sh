# kernel timeline of one headline solve (rocprofv3 --kernel-trace, per-launch rows kept)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
REPO=$(pwd)
out=$REPO/gpurun_out/r5/trace_${1:-on}
rm -rf "$out"; mkdir -p "$out"
shift
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$out" -o run -- python3 "$REPO/bench.py" --steps 1 --warmup 0 --no-cpu --no-copy-probe "$@" > "$out/stdout.log" 2>&1
rc=$?
echo "rc=$rc"
f=$(find "$out" -name '*kernel_trace.csv' | head -1)
python3 "$REPO/tools/trace_window.py" "$f" "${ANCHOR:-k_ilu_blocks_lds}" "${SKIP:-100}" "${COUNT:-24}" "${BEFORE:-4}" > "$out/window.txt" && rm -f "$f"
cat "$out/window.txt" | head -60
exit $rc
