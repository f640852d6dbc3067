#!/bin/bash
# round 6 final: the -m gpu suite in two halves (each under gpurun's 1,200 s), logs to gpurun_out/r6/
#   bash tools/r6_final_tests.sh 1|2
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out/r6
if [ "$1" = 1 ]; then files="tests/test_gpu_parity.py tests/test_gpu_amg.py"; else
  files=$(ls tests/test_*.py | grep -v "test_gpu_parity.py\|test_gpu_amg.py" | tr '\n' ' '); fi
timeout -k 10 1100 python -u -m pytest $files -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/r6/final_tests_$1.log 2>&1
rc=$?
grep -E "passed|failed|error" gpurun_out/r6/final_tests_$1.log | tail -3
grep -E "FAILED|ERROR" gpurun_out/r6/final_tests_$1.log | head
exit $rc
