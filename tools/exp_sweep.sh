# threads-per-workgroup of the LDS sweeps: auto vs forced 1024
set -o pipefail
for o in "" "--opt pls.sweep_tpb=1024"; do
  timeout -k 10 300 python -u bench.py --config footing-inexact --system fe --N 128 --steps 1 --warmup 0 --no-cpu --no-copy-probe --maxit 40 $o > gpurun_out/sw128.log 2>&1 || exit 1
  echo "footing N=128 40 its [$o] $(grep -o '"ms_per_step[^,]*' gpurun_out/sw128.log)"
  timeout -k 10 300 python -u bench.py --config footing-inexact --system fe --N 12 --steps 3 --no-cpu --no-copy-probe $o > gpurun_out/sw12.log 2>&1 || exit 1
  echo "footing N=12 [$o] $(grep -o '"value[^,]*' gpurun_out/sw12.log)"
  timeout -k 10 300 python -u bench.py --steps 5 --no-cpu --no-copy-probe $o > gpurun_out/swh.log 2>&1 || exit 1
  echo "headline [$o] $(grep -o '"value[^,]*' gpurun_out/swh.log)"
  for t in "" "--opt pls.sweep_tpb=256"; do timeout -k 10 300 python -u bench.py --system fe --N 12 --inner ilu --steps 3 --no-cpu --no-copy-probe $o $t > gpurun_out/swfe.log 2>&1 || exit 1; echo "fe N=12 ilu [$o $t] $(grep -o "\"value[^,]*" gpurun_out/swfe.log)"; done
done
