#!/bin/bash
# rocprofv3 per-dispatch kernel trace of a short bench run (for per-kernel
# breakdowns by launch order; no PMC counters).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
REPO=$(pwd)
mkdir -p gpurun_out/trace
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$REPO/gpurun_out/trace" -o run -- \
    python3 "$REPO/bench.py" --N "${N:-59}" --steps "${STEPS:-1}" --warmup 1 --no-cpu > "$REPO/gpurun_out/trace/stdout.log" 2>&1
rc=$?
echo "rocprofv3 rc=$rc"
find "$REPO/gpurun_out/trace" -name "*.csv" | head
exit $rc
