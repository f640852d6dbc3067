#!/bin/bash
# Rehearsal of bench.py's sharded path at 2/4/8 ranks on ONE GPU (ranks share
# the card through the host-staged gloo communicator, --comm host; RCCL
# refuses two ranks on one device).  Small global systems; each step has its
# own time limit and a failure stops the script.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out
export MASTER_ADDR=127.0.0.1
port=29531
for g in ${RANKS:-2 4 8}; do
    echo "=== ranks=$g"
    timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node "$g" --master-addr 127.0.0.1 \
        --master-port $port bench.py --gpus "$g" --N "${N:-12}" --steps 2 --warmup 1 --comm host --no-copy-probe \
        --scaling "${SCALING:-strong}" --no-cpu ${EXTRA:-} \
        > "gpurun_out/rehearse_${TAG:-}$g.log" 2>&1
    rc=$?
    echo "rc=$rc"; grep '^{' "gpurun_out/rehearse_${TAG:-}$g.log" | cut -c1-600 || tail -n 30 "gpurun_out/rehearse_${TAG:-}$g.log"
    [ $rc -eq 0 ] || exit $rc
    port=$((port + 1))
done
