#!/bin/bash
# One GPU-box session: parity tests, smoke, a short bench.  Each GPU step has
# its own time limit; a crash / timeout (exit not in {0,1}) stops the script.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out
step() {  # step <name> <seconds> <cmd...>
    local name=$1 secs=$2; shift 2
    echo "=== $name (limit ${secs}s)"
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"; tail -n 25 "gpurun_out/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
    return 0
}
case "${1:-all}" in
  tests) step pytest_gpu 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider ;;
  all)
    step pytest_gpu 900 python -m pytest tests -m gpu -q -p no:cacheprovider
    step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
    step bench_small 600 python bench.py --N 27 --steps 2 --warmup 1 --no-cpu
    ;;
  *) shift; step custom 1100 "$@" ;;
esac
