#!/bin/bash
# Secondary measurements: footing under a kernel trace, the AMG (inexact) and
# 3-way variants of the headline system.  Each step time-limited.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out/configs
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for v in "threeway:--pc-type 3-way --steps 3 --no-cpu" "amg-s-N27:--inner hypre --N 27 --steps 2 --no-cpu" "amg-s-N59:--inner hypre --steps 2 --no-cpu"; do
    name=${v%%:*}; args=${v#*:}
    timeout -k 10 400 python -u bench.py $args --no-copy-probe > gpurun_out/configs/$name.log 2>&1
    rc=$?; echo "$name rc=$rc"; cut -c1-400 gpurun_out/configs/$name.log | tail -n 3; [ $rc -eq 0 ] || exit $rc
done
