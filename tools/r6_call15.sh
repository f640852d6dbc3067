#!/bin/bash
# round 6: threshold pivoting's parallel fast path -- LU tests, harness, footing N=80 setup
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out/r6
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
    -k "sparse_lu or dense_lu or harness or exact" > gpurun_out/r6/lu_tests.log 2>&1
rc=$?; grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/r6/lu_tests.log | tail -n 40; [ $rc -eq 0 ] || exit $rc
timeout -k 10 260 python -u tools/robustness.py --problem footing --N 80 --pc undrained --set inexact \
    --opt pls.solver_time_limit=5 --opt pls.lu_view=1 > gpurun_out/r6/lu_view80_fast.log 2>&1 || exit $?
grep -E "dense lu|sparse lu" gpurun_out/r6/lu_view80_fast.log | cut -c1-500
grep '^{' gpurun_out/r6/lu_view80_fast.log | cut -c1-300
