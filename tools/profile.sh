#!/bin/bash
# rocprofv3 kernel-trace summary of a short bench run (no PMC counters here).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
mkdir -p gpurun_out/prof
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench -- \
    python3 bench.py --N "${N:-59}" --steps "${STEPS:-2}" --warmup 1 --no-cpu ${EXTRA:-} > gpurun_out/prof/bench_stdout.log 2>&1
rc=$?
echo "rocprofv3 rc=$rc"
find gpurun_out/prof -name "*stats*" | head
exit $rc
