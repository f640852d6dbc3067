#!/bin/bash
# Round-end: full GPU suite, smoke, headline bench (with CPU baseline), and a
# kernel trace of the headline for profiles/.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out/configs
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -n 1 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/configs/headline.log 2>&1
rc=$?; echo "bench rc=$rc"; grep '^{' gpurun_out/configs/headline.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
rm -rf gpurun_out/prof; mkdir -p gpurun_out/prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench -- \
    python3 bench.py --N 59 --steps 2 --warmup 1 --no-cpu > gpurun_out/prof/bench_stdout.log 2>&1
rc=$?; echo "rocprof rc=$rc"; exit $rc
