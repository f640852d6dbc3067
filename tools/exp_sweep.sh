# block-PC apply time on the assembled footing system: sweep workgroup size (auto vs 1024)
set -o pipefail
for N in 32 128; do
  for o in "" "pls.sweep_tpb=1024" "pls.sweep_tpb=256"; do
    timeout -k 10 200 python -u tools/pc_bench.py $N hypre $o || exit 1
  done
done
for o in "" "pls.sweep_tpb=1024"; do
  timeout -k 10 300 python -u bench.py --steps 5 --no-cpu --no-copy-probe ${o:+--opt $o} > gpurun_out/swh.log 2>&1 || exit 1
  echo "headline [$o] $(grep -o '"value[^,]*' gpurun_out/swh.log)"
  for t in "" "--opt pls.sweep_tpb=256"; do timeout -k 10 300 python -u bench.py --system fe --N 12 --inner ilu --steps 3 --no-cpu --no-copy-probe ${o:+--opt $o} $t > gpurun_out/swfe.log 2>&1 || exit 1; echo "fe N=12 ilu [$o $t] $(grep -o '"value[^,]*' gpurun_out/swfe.log)"; done
done
