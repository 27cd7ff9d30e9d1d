#!/bin/bash
# Quick round-3 pass: GPU tests (optional), bench (default + driver shape, no CPU baseline), the
# simulated strong scaling with and without the chain claim. usage: r3_quick.sh TAG [skip-tests]
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-q}
cd $R && mkdir -p gpurun_out/$TAG
O=$R/gpurun_out/$TAG
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu --maxfail=10 -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
  rc=$?
  grep -E "^FAILED|^ERROR" $O/gpu_tests.log | head -20
  tail -2 $O/gpu_tests.log
  # a failed test is reported, a crashed or hung run ends the call
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit 1; fi
fi
timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra > $O/bench_driver.log 2>&1 || exit 1
timeout -k 10 300 python scripts/strong_probe.py > $O/strong.txt 2>&1 || exit 1
PAMG_CHAIN_CLAIM=0 timeout -k 10 300 python scripts/strong_probe.py > $O/strong_noclaim.txt 2>&1 || exit 1
PAMG_CHAIN_CLAIM=0 timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra > $O/bench_noclaim.log 2>&1 || exit 1
grep -h "N=" $O/strong.txt $O/strong_noclaim.txt
for f in bench bench_driver bench_noclaim; do grep '^{' $O/$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['value'], d['roofline']['frac'])"; done
echo "all ok"
