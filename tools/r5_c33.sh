# footing N=40 inexact (the inner s-CG stops after ~2 its): which negative reason; and the N=10 harness parity tests
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5
timeout -k 10 300 python -u tools/robustness.py --problem footing --N 40 --pc "undrained" "undrained 3-way" --set inexact --out gpurun_out/r5/c33_footing40.jsonl > gpurun_out/r5/c33_footing40.log 2>&1 || { tail -20 gpurun_out/r5/c33_footing40.log; exit 1; }
python3 -c "
import json
for l in open('gpurun_out/r5/c33_footing40.jsonl'):
    d=json.loads(l); print(d['pc_type'], d['its'], d['reason'], {k:(v['its'],v['negative_reason'],v.get('last_negative')) for k,v in d['inner'].items()})"
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_harness.py > gpurun_out/r5/c33_harness.log 2>&1; rc=$?
tail -12 gpurun_out/r5/c33_harness.log
exit $rc
