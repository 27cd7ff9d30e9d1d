bash scripts/xc_check.sh xc2 || exit 1
for n in 2 4; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 2953$n bench.py --gpus $n --steps 20 --warmup 5 --comm detached > gpurun_out/xc2/mp_detached_$n.log 2>&1 || exit 1
  grep "^{" gpurun_out/xc2/mp_detached_$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); e=d['extra']; print($n, d['value'], e.get('halo_exchange1_vcycles_per_s'))"
done
