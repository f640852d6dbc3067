#!/bin/bash
# bench.py on the assembled swelling FE systems (lib/fe_swelling.py):
# configs[0] (2-D N=32, exact option set) with the 2-way and 3-way PCs, and
# the 3-D swelling system with ILU(0) blocks at a size the host assembles in
# seconds.  Output: gpurun_out/fe/*.log (one JSON line each).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out/fe
run() {
    local name=$1; shift
    timeout -k 10 300 python -u bench.py "$@" > gpurun_out/fe/$name.log 2>&1
    local rc=$?
    echo "$name rc=$rc"; grep '^{' gpurun_out/fe/$name.log | cut -c1-160
    return $rc
}
run exact2d_2way --config swelling2d-exact --system fe --steps 20 --warmup 2 --no-copy-probe &&
run exact2d_3way --config swelling2d-exact --system fe --pc-type "diagonal 3-way" --steps 20 --warmup 2 --no-copy-probe &&
run ilu3d_N12 --system fe --N 12 --inner ilu --steps 5 --warmup 1 --no-copy-probe --cpu-N 6 &&
run ilu3d_N20 --system fe --N 20 --inner ilu --steps 3 --warmup 1 --no-copy-probe --no-cpu
