#!/bin/bash
# Band-LU parity tests, then the footing configuration under a kernel trace.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out/configs
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread \
    -p no:cacheprovider -k "exact_lu or fieldsplit_fp" > gpurun_out/lu_band.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 4 gpurun_out/lu_band.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
rm -rf gpurun_out/prof_footing; mkdir -p gpurun_out/prof_footing
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_footing -o footing -- \
    python3 bench.py --config footing-inexact-ilu --steps 2 --warmup 1 --no-copy-probe \
    > gpurun_out/prof_footing/stdout.log 2>&1
rc=$?; echo "rocprof rc=$rc"; cut -c1-300 gpurun_out/prof_footing/stdout.log | tail -n 3
exit $rc
