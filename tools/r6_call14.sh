#!/bin/bash
# round 6: the window sweep's ring variant (tests), then the footing N=80 setup diagnosis
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out/r6
timeout -k 10 300 python -u -m pytest tests/test_gpu_sweeps.py -m gpu -x -v --timeout 120 --timeout-method thread \
    -p no:cacheprovider -k "window" > gpurun_out/r6/ring_tests.log 2>&1
rc=$?; tail -n 15 gpurun_out/r6/ring_tests.log; [ $rc -eq 0 ] || exit $rc
for v in "" "pls.lu_delay_rounds=0" "pls.lu_pivot_threshold=0"; do
    n=${v//[^a-z0-9]/_}
    timeout -k 10 260 python -u tools/robustness.py --problem footing --N 80 --pc undrained --set inexact \
        --opt pls.solver_time_limit=5 --opt pls.lu_view=1 ${v:+--opt $v} > gpurun_out/r6/lu_view80$n.log 2>&1 || exit $?
    grep -E "dense lu|sparse lu|setup|delayed" gpurun_out/r6/lu_view80$n.log | cut -c1-300
    grep '^{' gpurun_out/r6/lu_view80$n.log | cut -c1-400
done
