#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out/r6
timeout -k 10 120 python -u tools/r6_masked_check.py > gpurun_out/r6/masked_check.log 2>&1; rc=$?; cat gpurun_out/r6/masked_check.log | tail -3; [ $rc -eq 0 ] || exit $rc
bash tools/r6_sweep_ab.sh e160 swelling 160 || exit $?
bash tools/r6_sweep_ab.sh e160m swelling 160 pls.ring_probe=65536 || exit $?
