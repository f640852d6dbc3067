#!/bin/bash
# round 6: window ring variant A/B on the inexact cases whose hybrid-GS chunks exceed LDS
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out/r6
out=gpurun_out/r6/ring_ab.jsonl
for args in "swelling 160 diagonal" "footing 80 undrained"; do
  set -- $args
  for v in "pls.window_ring=-1" "pls.window_ring=0"; do
    timeout -k 10 200 python -u tools/robustness.py --problem $1 --N $2 --pc "$3" --set inexact \
        --opt pls.solver_time_limit=40 --opt pls.ilu_view=1 --opt $v --out $out \
        > gpurun_out/r6/ringab_$1_$2_${v//[^a-z0-9]/_}.log 2>&1 || exit $?
    echo "$1 $2 $v: $(grep -c 'sweep window-ring' gpurun_out/r6/ringab_$1_$2_${v//[^a-z0-9]/_}.log) ring-window PCs"
    tail -1 $out | cut -c1-420
  done
done
