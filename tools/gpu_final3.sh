#!/bin/bash
# Round-end: full GPU suite, smoke, headline bench (with CPU baseline), a
# kernel trace of the headline and of the assembled 3-D N=12 swelling solve
# (whole-block ILU(0), y-resident sweep) for profiles/.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
REPO=$(pwd)
mkdir -p gpurun_out/configs gpurun_out/fe
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -n 1 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/configs/headline.log 2>&1
rc=$?; echo "bench rc=$rc"; grep '^{' gpurun_out/configs/headline.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
rm -rf "$REPO/gpurun_out/prof" "$REPO/gpurun_out/prof_fe"; mkdir -p "$REPO/gpurun_out/prof" "$REPO/gpurun_out/prof_fe"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$REPO/gpurun_out/prof" -o bench -- \
    python3 "$REPO/bench.py" --N 59 --steps 2 --warmup 1 --no-cpu > "$REPO/gpurun_out/prof/bench_stdout.log" 2>&1
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$REPO/gpurun_out/prof_fe" -o fe -- \
    python3 "$REPO/bench.py" --system fe --N 12 --inner ilu --steps 2 --warmup 1 --no-cpu --no-copy-probe \
    > "$REPO/gpurun_out/prof_fe/fe_stdout.log" 2>&1
rc=$?; echo "rocprof fe rc=$rc"; exit $rc
