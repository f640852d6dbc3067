#!/bin/bash
# One inexact harness case under several library options (the level-0 hybrid
# Gauss-Seidel sweep variants), each cut at TL seconds: s-CG iterations per second.
#   bash tools/r6_sweep_variants.sh <problem> <N> <pc type> <TL> "<opts1>" "<opts2>" ...
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
prob=$1; N=$2; pc=$3; TL=$4; shift 4
out=gpurun_out/variants_${prob}_${N}.jsonl
rm -f $out
for o in "$@"; do
  args=(--opt pls.solver_time_limit=$TL --opt pls.ilu_view=1)
  for kv in $o; do args+=(--opt "$kv"); done
  echo "=== variant: $o"
  timeout -k 10 $((TL + 120)) python -u tools/robustness.py --problem $prob --N $N --pc "$pc" --set inexact \
      "${args[@]}" --out $out > gpurun_out/variant.log 2>&1
  rc=$?
  grep "pls ilu\]" gpurun_out/variant.log | sort | uniq -c | head -12
  tail -1 $out | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); s=d['inner'].get('s_',{}); print('its',d['its'],'solve_s',d['solve_s'],'s_its',s.get('its'),'s_its_per_s',round(s.get('its',0)/d['solve_s'],1))"
  [ $rc -eq 0 ] || exit $rc
done
