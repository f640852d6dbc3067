cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5
export OMP_NUM_THREADS=2
timeout -k 10 600 python -u tools/g8_n27.py 8 27 solve_first > gpurun_out/r5/g8n27sf.log 2>&1; rc=$?
tail -1 gpurun_out/r5/g8n27sf.log; [ $rc -eq 0 ] || exit $rc
unset OMP_NUM_THREADS
rm -f gpurun_out/r5/rob10.jsonl
timeout -k 10 500 python -u tools/robustness.py --problem swelling --N 10 --pc "diagonal" "diagonal 3-way" --oracle --out gpurun_out/r5/rob10.jsonl > gpurun_out/r5/rob10_sw.log 2>&1; rc=$?
tail -2 gpurun_out/r5/rob10_sw.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u tools/robustness.py --problem footing --N 10 --pc "undrained" "undrained 3-way" --oracle --out gpurun_out/r5/rob10.jsonl > gpurun_out/r5/rob10_ft.log 2>&1; rc=$?
tail -2 gpurun_out/r5/rob10_ft.log | cut -c1-300; exit $rc
