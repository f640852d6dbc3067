#!/bin/bash
# round 6: window tests, level-0 sweep timing (kernel trace), then s-CG iterations/s without the profiler
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out/r6
timeout -k 10 400 python -u -m pytest tests/test_gpu_sweeps.py tests/test_gpu_harness.py -m gpu -x -v --timeout 120 --timeout-method thread \
    -p no:cacheprovider -k "window or harness" > gpurun_out/r6/win_tests.log 2>&1
rc=$?; grep -E "passed|failed" gpurun_out/r6/win_tests.log | tail -n 2; [ $rc -eq 0 ] || exit $rc
bash tools/r6_sweep_ab.sh g80 swelling 80 || exit $?
bash tools/r6_sweep_ab.sh g160 swelling 160 || exit $?
for N in 80 160; do
  timeout -k 10 300 python -u tools/robustness.py --problem swelling --N $N --pc diagonal --set inexact \
      --opt pls.solver_time_limit=5 --opt s_ksp_max_it=2000 --out gpurun_out/r6/rate.jsonl > gpurun_out/r6/rate_$N.log 2>&1 || exit $?
  python3 -c "
import json; d=[json.loads(l) for l in open('gpurun_out/r6/rate.jsonl')][-1]; s=d['inner']['s_']
print('swelling N=%d inexact: %d s-CG its in %.2f s solve: %.0f its/s, %.3f ms/it' % (d['N'], s['its'], d['solve_s'], s['its']/d['solve_s'], 1e3*d['solve_s']/s['its']))"
done
