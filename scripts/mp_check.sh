#!/bin/bash
# Multi-process orchestration of bench.py on a one-GPU box: 2 ranks, detached partitions
# (no RCCL: it refuses two ranks on one GPU), the driver's launch line otherwise.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 2 --comm detached > gpurun_out/mp_check.log 2>&1
rc=$?
echo "exit $rc"
exit $rc
