# footing.py's own option set (classical AMG) at growing N: outer its / time, default chunks vs one chunk
for N in 16 24 32; do
for o in pls.hypre_relax_chunks=256 pls.hypre_relax_chunks=1; do
  timeout -k 10 300 python -u bench.py --config footing-inexact --system fe --N $N --steps 1 --warmup 0 --no-cpu --no-copy-probe --opt $o > gpurun_out/f_${N}_$o.log 2>&1 || exit 1
  echo "N=$N $o $(grep -o '"its_per_solve[^,]*' gpurun_out/f_${N}_$o.log) $(grep -o '"ms_per_step[^,]*' gpurun_out/f_${N}_$o.log) $(grep -o '"reasons[^]]*' gpurun_out/f_${N}_$o.log)"
done; done
