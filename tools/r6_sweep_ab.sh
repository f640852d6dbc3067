#!/bin/bash
# round 6: the level-0 hybrid-GS sweep per launch (the AMG smoother's np=8 chunks), from the
# kernel trace: launches of the ILU sweep kernels with grid = 8 workgroups (the level-0 chunks)
#   bash tools/r6_sweep_ab.sh <name> <problem> <N> [--opt k=v ...]
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
name=$1 prob=$2 N=$3; shift 3
bash tools/prof_inexact.sh r6/$name $prob $N diagonal 5 s_ksp_max_it=300 pls.ilu_view=1 "$@" > /dev/null 2>&1 || exit $?
echo "== $name $*: $(grep 'pls ilu' gpurun_out/r6/$name/stdout.log | grep -v 'n 1[0-9] ' | cut -c1-160)"
python3 - gpurun_out/r6/$name <<'PY'
import csv, sys, collections
d = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1] + "/trace_head.csv")):
    if "k_ilu_blocks" in r["Kernel_Name"]:
        d[(r["Kernel_Name"][:48], int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"]))].append(
            (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for (k, g), v in sorted(d.items()):
    v.sort()
    print(f"   {k} grid {g}: {len(v)} launches, mean {sum(v)/len(v):.1f} us, median {v[len(v)//2]:.1f} us")
PY
rm -f gpurun_out/r6/$name/trace_head.csv
