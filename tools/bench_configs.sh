#!/bin/bash
# bench.py on every BASELINE.json configuration that fits one GPU (the
# headline is configs[1] at N=59; these lines feed DESIGN.md's config table).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out/configs
run() {  # run <name> <args...>
    local name=$1; shift
    echo "=== $name: $*"
    timeout -k 10 400 python bench.py "$@" > "gpurun_out/configs/$name.log" 2>&1 &
    local pid=$!
    while kill -0 $pid 2>/dev/null; do sleep 20; echo "  ... $name running"; done
    wait $pid
    local rc=$?
    echo "rc=$rc"; grep '^{' "gpurun_out/configs/$name.log" | cut -c1-900 || tail -n 20 "gpurun_out/configs/$name.log"
    [ $rc -eq 0 ] || exit $rc
}
run headline --steps 5
run swelling2d-exact --config swelling2d-exact --steps 3 --no-copy-probe
run footing-inexact-ilu --config footing-inexact-ilu --steps 2 --no-copy-probe
run aar-m5 --config aar-m5 --steps 2 --no-copy-probe
run swelling3d-N64 --config swelling3d-bjacobi --N 64 --steps 2 --no-copy-probe --no-cpu
