#!/bin/bash
# Round-3 evidence pass: GPU tests, bench (default and the driver's shape), the roofline sweep
# kernels under rocprofv3 (kernel stats, FETCH/WRITE PMC passes), the simulated strong scaling
# (in-tree + scripts/ablibs), the 2-rank detached orchestration check. usage: r3_check.sh TAG [skip-tests]
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r3}
cd $R && mkdir -p gpurun_out/$TAG
O=$R/gpurun_out/$TAG
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -30 $O/gpu_tests.log; exit 1; }
  tail -3 $O/gpu_tests.log
fi
timeout -k 10 500 python bench.py > $O/bench.log 2>&1 || { echo "bench failed"; tail -20 $O/bench.log; exit 1; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra > $O/bench_driver.log 2>&1 || exit 1
timeout -k 10 300 python scripts/sweep_prof.py > $O/sweep.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_sweep -o run -- python3 $R/scripts/sweep_prof.py > $O/prof_sweep.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc_sweep_fetch -o run -- python3 $R/scripts/sweep_prof.py 3 > $O/pmc_sweep_fetch.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmc_sweep_write -o run -- python3 $R/scripts/sweep_prof.py 3 > $O/pmc_sweep_write.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_bench -o run -- python3 $R/bench.py --no-cpu-baseline --no-extra > $O/prof_bench.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc_res_fetch -o run -- python3 $R/bench.py --steps 20 --warmup 1 --no-cpu-baseline --no-extra > $O/pmc_res_fetch.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmc_res_write -o run -- python3 $R/bench.py --steps 20 --warmup 1 --no-cpu-baseline --no-extra > $O/pmc_res_write.log 2>&1 || exit 1
cd $R
echo "== in-tree" > $O/strong.txt
timeout -k 10 300 python scripts/strong_probe.py >> $O/strong.txt 2>&1 || exit 1
for f in scripts/ablibs/*.so; do
  [ -e "$f" ] || continue
  echo "== $(basename $f)" >> $O/strong.txt
  PAMG_LIB=$PWD/$f timeout -k 10 300 python scripts/strong_probe.py >> $O/strong.txt 2>&1 || exit 1
done
for n in 2 4; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port 2953$n bench.py --gpus $n --steps 20 --warmup 5 --comm detached > $O/mp_detached_$n.log 2>&1 || exit 1
done
echo "all ok"
