# robustness_2d.sh's slow inexact cases, each stopped by a wall-clock limit on
# the outer solve (pls.solver_time_limit; reason -100) so its iteration count,
# residual and inner-solver statistics at the cutoff are recorded
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5
out=gpurun_out/r5/robustness_slow.jsonl
TL=${TL:-240}
while [ $# -gt 0 ]; do
  prob=$1; N=$2; pc=$3; shift 3
  timeout -k 10 $((TL + 240)) python -u tools/robustness.py --problem $prob --N $N --pc "$pc" --set inexact \
      --opt pls.solver_time_limit=$TL --out $out > gpurun_out/r5/robx_${prob}_${N}_${pc// /_}.log 2>&1
  rc=$?
  echo "$prob N=$N '$pc' rc=$rc $(tail -1 $out | cut -c1-220)"
  [ $rc -eq 0 ] || exit $rc
done
