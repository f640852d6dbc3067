cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5
export OMP_NUM_THREADS=2
timeout -k 10 1000 python -u tools/g8_n27.py 8 27 solve_first > gpurun_out/r5/g8n27sf.log 2>&1; rc=$?
tail -3 gpurun_out/r5/g8n27sf.log; exit $rc
