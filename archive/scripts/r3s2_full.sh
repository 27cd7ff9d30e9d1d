#!/bin/bash
# Session-2 evidence pass: all GPU tests, the bench (default, the driver's shape), the simulated strong
# scaling, 2- and 4-rank detached benches, the face probe. usage: r3s2_full.sh TAG [skip-tests]
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/${1:-full}; mkdir -p $O
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu --maxfail=5 -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
  rc=$?
  grep -E "^FAILED|^ERROR" $O/gpu_tests.log | head -20; tail -2 $O/gpu_tests.log
  if [ $rc -ne 0 ]; then echo "tests rc $rc"; exit 1; fi
fi
timeout -k 10 400 python bench.py --no-cpu-baseline > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra > $O/bench_driver.log 2>&1 || exit 1
timeout -k 10 300 python scripts/strong_probe.py > $O/strong.txt 2>&1 || exit 1
PAMG_RES_W4=0 timeout -k 10 300 python scripts/strong_probe.py > $O/strong_w3.txt 2>&1 || exit 1
for n in 2 4; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port 2953$n bench.py --gpus $n --steps 20 --warmup 5 --comm detached > $O/mp_detached_$n.log 2>&1 || exit 1
done
grep -h "N=" $O/strong.txt $O/strong_w3.txt | cut -c1-200
for f in bench bench_driver mp_detached_2 mp_detached_4; do grep '^{' $O/$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); e=d.get('extra',{}); print('$f', d['value'], d['roofline']['frac'], e.get('halo_exchange1_vcycles_per_s'), (e.get('op1') or {}).get('vcycles_per_s'))"; done
echo "all ok"
