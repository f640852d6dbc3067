#!/bin/bash
# Round-end check: full GPU parity suite, smoke, headline bench, footing under
# a kernel trace.  Stops at the first failing step.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out/configs
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -n 1 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/configs/headline.log 2>&1
rc=$?; echo "bench rc=$rc"; grep '^{' gpurun_out/configs/headline.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
rm -rf gpurun_out/prof_footing; mkdir -p gpurun_out/prof_footing
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_footing -o footing -- \
    python3 bench.py --config footing-inexact-ilu --steps 2 --warmup 1 --no-copy-probe \
    > gpurun_out/prof_footing/stdout.log 2>&1
rc=$?; echo "footing rocprof rc=$rc"; exit $rc
