#!/bin/bash
# Overlapped halo exchange: distributed parity tests, then the 2-rank sharded
# rehearsal (N=74 global, ranks sharing the GPU, host-staged communicator)
# with and without the overlap.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out
export MASTER_ADDR=127.0.0.1
timeout -k 10 900 python -u -m pytest tests/test_dist_gpu.py -x -v --timeout 600 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/dist_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 gpurun_out/dist_tests.log; [ $rc -eq 0 ] || exit $rc
port=29541
for ov in 1 0; do
    timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
        --master-port $port bench.py --gpus 2 --N 59 --steps 2 --warmup 1 --comm host --no-copy-probe \
        --opt pls.halo_overlap=$ov > gpurun_out/overlap_$ov.log 2>&1
    rc=$?; echo "overlap=$ov rc=$rc $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"its_per_solve": [0-9.]*\|"spmv_total": [0-9.]*' gpurun_out/overlap_$ov.log | tr '\n' ' ')"
    [ $rc -eq 0 ] || exit $rc
    port=$((port + 1))
done
