#!/bin/bash
# Full GPU session: parity suite, smoke, every bench configuration, a kernel
# trace of the footing configuration.  Stops at the first failing step.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 4 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -n 2 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
bash tools/bench_configs.sh || exit $?
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/prof_footing
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_footing -o footing -- \
    python3 bench.py --config footing-inexact-ilu --steps 1 --warmup 1 --no-cpu --no-copy-probe \
    > gpurun_out/prof_footing/stdout.log 2>&1
echo "rocprof rc=$?"
