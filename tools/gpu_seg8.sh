#!/bin/bash
# 8-segment D16 layout: parity tests, the 2-rank sharded rehearsal (N=74 global),
# and the single-GPU headline for regressions.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out/configs
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_dist_gpu.py tests/test_gpu_large.py -x -v \
    --timeout 300 --timeout-method thread -p no:cacheprovider -k "spmv or seg8 or dist or full_size" \
    > gpurun_out/seg8_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 gpurun_out/seg8_tests.log; [ $rc -eq 0 ] || exit $rc
RANKS=2 N=59 bash tools/rehearse_dist.sh || exit $?
grep -o '"layout": "[^"]*"\|"achieved": [0-9.]*\|"isolated_spmv_gbs": [0-9.]*\|"ms_per_step": [0-9.]*\|"its_per_solve": [0-9.]*' gpurun_out/rehearse_2.log | tr '\n' ' '; echo
timeout -k 10 400 python -u bench.py --no-cpu --steps 3 > gpurun_out/configs/headline_seg.log 2>&1
rc=$?; echo "bench rc=$rc"; grep -o '"value": [0-9.]*\|"achieved": [0-9.]*\|"layout": "[^"]*"' gpurun_out/configs/headline_seg.log | tr '\n' ' '
exit $rc
