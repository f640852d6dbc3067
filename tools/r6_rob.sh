#!/bin/bash
# robustness_2d.sh's cases (tools/robustness.py), each outer solve cut at TL
# seconds (pls.solver_time_limit; reason -100 = cut, not a PETSc reason).
#   TL=240 SET=inexact bash tools/r6_rob.sh <problem> <N> <pc type> [<problem> <N> <pc type> ...]
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out/r6
out=gpurun_out/r6/robustness.jsonl
TL=${TL:-240}
SET=${SET:-inexact}
while [ $# -gt 0 ]; do
  prob=$1; N=$2; pc=$3; shift 3
  timeout -k 10 $((TL + 300)) python -u tools/robustness.py --problem $prob --N $N --pc "$pc" --set $SET \
      --opt pls.solver_time_limit=$TL --out $out > gpurun_out/r6/rob_${prob}_${N}_${pc// /_}_${SET}.log 2>&1
  rc=$?
  echo "$prob N=$N '$pc' $SET rc=$rc $(tail -1 $out | cut -c1-240)"
  [ $rc -eq 0 ] || exit $rc
done
