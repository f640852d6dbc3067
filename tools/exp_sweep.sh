set -o pipefail
for N in 32 128; do
  for o in "pls.sweep_rr=0" ""; do
    timeout -k 10 200 python -u tools/pc_bench.py $N hypre $o || exit 1
  done
done
timeout -k 10 200 python -u tools/pc_bench.py 128 hypre pls.sweep_profile=1 2>&1 | grep "blk\|sweep" | head -6
