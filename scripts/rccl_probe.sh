#!/bin/bash
# 2 ranks through torch.distributed.run; on a 1-GPU box both ranks map to device 0.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 2 > gpurun_out/rccl_probe.log 2>&1
echo "exit $?"
