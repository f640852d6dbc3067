#!/bin/bash
# One parameterised GPU-box session (replaces the round-1 one-off scripts).
#
#   bash tools/gpu.sh <step> [<step> ...]
#
# steps (run in order; each has its own time limit; the first failure,
# timeout or crash ends the script -- no GPU step runs after it):
#   tests[=<pytest -k expr>]   the -m gpu suite (optionally a subset)
#   smoke                       __graft_entry__.smoke()
#   bench                       the headline bench line (default flags)
#   prof                        rocprofv3 --kernel-trace --stats of the headline
#   prof_fe                     same for the assembled 3-D N=12 whole-block ILU solve
#   prof_fe24                   same at 3-D N=24 (721,519 DoF; the FE SpMV layout), 10 its
#   prof_footing                same for configs[2] (footing-inexact-ilu, band-LU Schur block)
#   footing                     configs[2] bench on the assembled footing system (N=128)
#   prof_footing_fe             rocprofv3 of that solve
#   footing128 / prof_footing128  configs[2] at N=128 with footing.py's own set (classical AMG, sparse LU)
#   prof_amg                    same for the classical AMG (-pc_type hypre) on the s block, 3-D N=27
#   prof_amg59                  same at the metric's N=59
#   configs                     bench on every BASELINE config that fits one GPU
#   fe                          bench on the assembled swelling systems
#   pmc                         FETCH_SIZE / WRITE_SIZE passes (tools/pmc.sh)
#   custom:<name>:<cmd>         any command, output in gpurun_out/<name>.log
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
REPO=$(pwd)
mkdir -p gpurun_out/configs gpurun_out/fe

run() {  # run <log> <seconds> <cmd...>   (progress line every 30 s)
    local log=$1 secs=$2; shift 2
    echo "=== $log (limit ${secs}s): $*"
    timeout -k 10 "$secs" "$@" > "$REPO/gpurun_out/$log.log" 2>&1 &
    local pid=$!
    while kill -0 $pid 2>/dev/null; do sleep 30; kill -0 $pid 2>/dev/null && echo "  ... $log running"; done
    wait $pid
    local rc=$?
    echo "=== $log rc=$rc"
    grep '^{' "$REPO/gpurun_out/$log.log" | cut -c1-600
    tail -n 4 "$REPO/gpurun_out/$log.log"
    if [ $rc -ne 0 ]; then echo "STOP after $log (rc=$rc)"; exit $rc; fi
}

prof() {  # prof <dir> <bench args...>
    local dir=$1; shift
    rm -rf "$REPO/gpurun_out/$dir"; mkdir -p "$REPO/gpurun_out/$dir"
    (cd /tmp && export TMPDIR=/tmp &&
     run "$dir/stdout" 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$REPO/gpurun_out/$dir" -o run -- \
         python3 "$REPO/bench.py" "$@") || exit $?
    rm -f "$REPO/gpurun_out/$dir"/run_kernel_trace.csv  # per-launch rows: too large to copy back
}

for s in "$@"; do
    case "$s" in
      tests) run pytest_gpu 1500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider ;;
      tests=*) run pytest_gpu_sub 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
                   -p no:cacheprovider -k "${s#tests=}" ;;
      smoke) run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" ;;
      bench) run configs/headline 500 python -u bench.py ;;
      prof) prof prof --steps 2 --warmup 1 --no-cpu ;;
      prof_footing) prof prof_footing --config footing-inexact-ilu --steps 3 --warmup 1 --no-cpu --no-copy-probe ;;
      prof_amg) prof prof_amg --N 27 --inner hypre --steps 2 --warmup 1 --no-cpu --no-copy-probe ;;
      prof_amg59) prof prof_amg59 --inner hypre --steps 1 --warmup 1 --no-cpu --no-copy-probe ;;
      prof_fe) prof prof_fe --system fe --N 12 --inner ilu --steps 2 --warmup 1 --no-cpu --no-copy-probe ;;
      prof_fe24) prof prof_fe24 --system fe --N 24 --inner ilu --steps 1 --warmup 1 --maxit 10 --no-cpu --no-copy-probe ;;
      configs)
        run configs/swelling2d-exact 400 python -u bench.py --config swelling2d-exact --steps 3 --no-copy-probe
        run configs/footing-inexact-ilu 400 python -u bench.py --config footing-inexact-ilu --steps 2 --no-copy-probe
        run configs/aar-m5 400 python -u bench.py --config aar-m5 --steps 2 --no-copy-probe
        run configs/swelling3d-N64 400 python -u bench.py --config swelling3d-bjacobi --N 64 --steps 2 --no-copy-probe --no-cpu ;;
      fe)
        run fe/exact2d_2way 300 python -u bench.py --config swelling2d-exact --system fe --steps 20 --warmup 2 --no-copy-probe
        run fe/exact2d_3way 300 python -u bench.py --config swelling2d-exact --system fe --pc-type "diagonal 3-way" --steps 20 --warmup 2 --no-copy-probe
        run fe/ilu3d_N12 300 python -u bench.py --system fe --N 12 --inner ilu --steps 5 --warmup 1 --no-copy-probe --cpu-N 6
        run fe/ilu3d_N20 300 python -u bench.py --system fe --N 20 --inner ilu --steps 3 --warmup 1 --no-copy-probe --no-cpu ;;
      footing)  # configs[2] on the assembled footing system (lib/fe_footing.py)
        run fe/footing_N128 600 python -u bench.py --config footing-inexact-ilu --system fe --steps 2 --warmup 1 --no-copy-probe ;;
      prof_footing_fe) prof prof_footing_fe --config footing-inexact-ilu --system fe --steps 2 --warmup 1 --no-cpu --no-copy-probe ;;
      prof_footing_amg) prof prof_footing_amg --config footing-inexact --system fe --N 12 --steps 1 --warmup 0 --no-cpu --no-copy-probe ;;
      prof_footing128) prof prof_footing128 --config footing-inexact --system fe --N 128 --steps 1 --warmup 0 --no-cpu --no-copy-probe --maxit 40 ;;
      footing128) run fe/footing_amg_N128 1000 python -u bench.py --config footing-inexact --system fe --N 128 --steps 1 --warmup 0 --no-copy-probe --opt pls.lu_view=1 --opt pls.amg_view=1 --opt pls.ksp_stats=1 ;;
      pmc) run pmc 1300 bash tools/pmc.sh ;;
      custom:*) rest=${s#custom:}; name=${rest%%:*}; cmd=${rest#*:}; run "$name" 1100 bash -c "$cmd" ;;
      *) echo "unknown step $s"; exit 2 ;;
    esac
done
