#!/bin/bash
# round 6: swelling N=160 inexact, 1,000 s-CG its per solve: kernel stats, default vs the forced window sweeps
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
bash tools/prof_inexact.sh r6/prof160 swelling 160 diagonal 5 s_ksp_max_it=1000 pls.ilu_view=1 || exit $?
bash tools/prof_inexact.sh r6/prof160w swelling 160 diagonal 5 s_ksp_max_it=1000 pls.ilu_view=1 pls.window_depth=3 || exit $?
for d in prof160 prof160w; do
  grep "pls ilu" gpurun_out/r6/$d/stdout.log | sort | uniq -c
  grep '^{' gpurun_out/r6/$d/case.jsonl | cut -c1-400
  python3 - gpurun_out/r6/$d <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:14]:
    print(f'{float(r["TotalDurationNs"])/1e6:10.1f} ms {int(r["Calls"]):8d} {float(r["AverageNs"])/1e3:9.1f} us  {r["Name"][:90]}')
PY
done
