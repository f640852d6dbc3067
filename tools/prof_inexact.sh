#!/bin/bash
# rocprofv3 kernel trace of one of robustness_2d.sh's inexact cases (the
# reference's harness, tools/robustness.py), the outer solve cut at TL seconds.
#   bash tools/prof_inexact.sh <name> <problem> <N> <pc type> [TL] [extra --opt k=v ...]
# Writes gpurun_out/<name>/ (kernel stats CSV, a per-launch trace trimmed to
# its first 60,000 launches) and the case's JSON line.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
REPO=$(pwd)
name=$1; prob=$2; N=$3; pc=$4; TL=${5:-10}; shift 5
out="$REPO/gpurun_out/$name"
rm -rf "$out"; mkdir -p "$out"
opts=()
for kv in "$@"; do opts+=(--opt "$kv"); done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 $((TL + 200)) rocprofv3 --kernel-trace --stats --output-format csv -d "$out" -o run -- \
    python3 -u "$REPO/tools/robustness.py" --problem "$prob" --N "$N" --pc "$pc" --set inexact \
    --opt pls.solver_time_limit=$TL --opt pls.ksp_stats=1 "${opts[@]}" --out "$out/case.jsonl" > "$out/stdout.log" 2>&1
rc=$?
f=$(find "$out" -name "*kernel_trace.csv" | head -1)
if [ -n "$f" ]; then head -n 60001 "$f" > "$out/trace_head.csv"; rm -f "$f"; fi
tail -3 "$out/stdout.log"
exit $rc
