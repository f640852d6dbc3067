#!/bin/bash
# round 6: s-CG iterations per second of the reference's inexact set (swelling 2-way, np=8 semantics), no profiler
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out/r6
for N in 80 160; do
  timeout -k 10 300 python -u tools/robustness.py --problem swelling --N $N --pc diagonal --set inexact \
      --opt pls.solver_time_limit=5 --opt s_ksp_max_it=2000 --out gpurun_out/r6/rate.jsonl > gpurun_out/r6/rate_$N.log 2>&1 || exit $?
done
python3 -c "
import json
for l in open('gpurun_out/r6/rate.jsonl'):
    d=json.loads(l); s=d['inner']['s_']
    print('swelling N=%d inexact: %d s-CG its in %.2f s solve: %.0f its/s, %.3f ms/it' % (d['N'], s['its'], d['solve_s'], s['its']/d['solve_s'], 1e3*d['solve_s']/s['its']))"
