#!/bin/bash
# round 6: robustness rows (TL 280 s) then the swelling N=160 s-CG rate
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
SET=inexact TL=280 bash tools/r6_rob.sh "$@" || exit $?
timeout -k 10 300 python -u tools/robustness.py --problem swelling --N 160 --pc diagonal --set inexact \
    --opt pls.solver_time_limit=5 --opt s_ksp_max_it=2000 --out gpurun_out/r6/rate.jsonl > gpurun_out/r6/rate_160.log 2>&1 || exit $?
python3 -c "
import json; d=[json.loads(l) for l in open('gpurun_out/r6/rate.jsonl')][-1]; s=d['inner']['s_']
print('swelling N=%d inexact: %d s-CG its in %.2f s solve: %.0f its/s, %.3f ms/it' % (d['N'], s['its'], d['solve_s'], s['its']/d['solve_s'], 1e3*d['solve_s']/s['its']))"
