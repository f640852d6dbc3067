# footing.py's own option set (classical AMG): inner iteration statistics at growing N
for N in 16 32 64 128; do
  timeout -k 10 240 python -u bench.py --config footing-inexact --system fe --N $N --steps 1 --warmup 0 --no-cpu --no-copy-probe --maxit 40 --opt pls.ksp_stats=1 $EXTRA > gpurun_out/fstat_$N.log 2>&1 || { echo "N=$N failed/timeout"; tail -3 gpurun_out/fstat_$N.log; exit 1; }
  echo "N=$N $(grep -o '"its_per_solve[^,]*' gpurun_out/fstat_$N.log) $(grep -o '"ms_per_step[^,]*' gpurun_out/fstat_$N.log)"
  grep '^\[ksp' gpurun_out/fstat_$N.log
done
