#!/bin/bash
# A/B the headline bench over library options (each line of $@ one option set,
# "" = defaults), interleaved twice; one JSON summary line per run.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
out=gpurun_out/ab.log
: > $out
for rep in 1 2; do
  for o in "$@"; do
    args=()
    for kv in $o; do args+=(--opt "$kv"); done
    timeout -k 10 300 python -u bench.py --no-cpu --no-copy-probe "${args[@]}" > gpurun_out/ab_run.log 2>&1
    rc=$?
    v=$(grep '^{' gpurun_out/ab_run.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value'],2), round(d['ms_per_step'],1))")
    echo "rep $rep [$o] -> $v" | tee -a $out
    [ $rc -eq 0 ] || exit $rc
  done
done
