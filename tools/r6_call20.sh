#!/bin/bash
# round 6: where the ring window sweep's time goes -- N=80 LDS window vs the ring variant on the same
# chunks, and N=160 with the stores removed / out of range (timing probes)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
run() {  # name problem N extra...
  local name=$1 prob=$2 N=$3; shift 3
  bash tools/prof_inexact.sh r6/$name $prob $N diagonal 5 s_ksp_max_it=300 pls.ilu_view=1 "$@" > /dev/null 2>&1 || return $?
  echo "== $name $*: $(grep 'pls ilu' gpurun_out/r6/$name/stdout.log | grep -v 'n 14 ' | cut -c1-160)"
  python3 - gpurun_out/r6/$name <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "k_ilu_blocks" in r["Name"] and float(r["AverageNs"]) > 50000:
        print(f'   {int(r["Calls"]):6d} x {float(r["AverageNs"])/1e3:8.1f} us  {r["Name"][:60]}')
PY
}
run a80 swelling 80 || exit $?
run a80r swelling 80 pls.window_ring=1 || exit $?
run a160 swelling 160 || exit $?
run a160ns swelling 160 pls.ring_probe=2048 || exit $?
run a160oor swelling 160 pls.ring_probe=4096 || exit $?
