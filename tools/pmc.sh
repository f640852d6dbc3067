#!/bin/bash
# HBM traffic of the bench's kernels from PMC counters (MI355X_MICROARCH.md,
# HBM section): FETCH_SIZE and WRITE_SIZE in separate passes (they do not fit
# one pass), each with --kernel-trace only.  tools/pmc_summary.py turns the
# per-dispatch counters into per-launch bytes (FETCH_SIZE x 2 on gfx950).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
REPO=$(pwd)
mkdir -p gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $c --kernel-trace --output-format csv -d "$REPO/gpurun_out/pmc/$c" -o run -- \
      python3 "$REPO/bench.py" --N "${N:-59}" --steps 1 --warmup 0 --no-cpu > "$REPO/gpurun_out/pmc/$c.log" 2>&1 || exit $?
done
cd "$REPO" && python3 tools/pmc_summary.py gpurun_out/pmc
