# robustness_2d.sh on the device (tools/robustness.py), one option set / problem per call
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5
out=gpurun_out/r5/robustness_$1_$2.jsonl
rm -f $out
shift 0
prob=$1; set_=$2; shift 2
if [ "$prob" = swelling ]; then pcs=("diagonal" "diagonal 3-way"); Ns=${NS:-"10 20 40 80 160"}; else pcs=("undrained" "undrained 3-way"); Ns=${NS:-"10 20 40 80"}; fi
for N in $Ns; do for pc in "${pcs[@]}"; do
  timeout -k 10 ${TLIM:-600} python -u tools/robustness.py --problem $prob --N $N --pc "$pc" --set $set_ --out $out "$@" > gpurun_out/r5/rob_${prob}_${set_}_${N}.log 2>&1
  rc=$?
  echo "$prob $set_ N=$N '$pc' rc=$rc $(tail -1 $out | cut -c1-200)"
  [ $rc -eq 0 ] || exit $rc
done; done
