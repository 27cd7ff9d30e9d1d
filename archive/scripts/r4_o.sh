#!/bin/bash
# bench.py's N-rank path at HEAD, 2 and 4 detached ranks sharing the one GPU (no RCCL: orchestration,
# barrier and max-over-ranks timing; the driver's node runs the RCCL form)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/r4o; mkdir -p $O
for n in 2 4; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port 2963$n bench.py --gpus $n --steps 20 --warmup 5 --comm detached > $O/mp_detached_$n.log 2>&1 || { tail -20 $O/mp_detached_$n.log; exit 1; }
  grep '^{' $O/mp_detached_$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print($n, d['value'], d['ms_per_step'], d['n_gpus'], d['extra'].get('rank_ms_per_step'))"
done
echo "all ok"
