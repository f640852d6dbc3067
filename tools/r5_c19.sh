cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5
timeout -k 10 840 python -u tools/robustness.py --problem swelling --N 80 --pc "diagonal 3-way" --set inexact --monitor --opt pls.ksp_stats=1 --out gpurun_out/r5/rob_sw80_3way.jsonl > gpurun_out/r5/rob_sw80_3way.log 2>&1
rc=$?; echo rc=$rc; grep -c "KSP Residual" gpurun_out/r5/rob_sw80_3way.log; tail -4 gpurun_out/r5/rob_sw80_3way.log | cut -c1-400; exit $rc
