#!/bin/bash
# Round-3 final evidence: GPU tests, smoke, the bench (default and the driver's shape, with the CPU
# baseline), rocprofv3 kernel stats of the bench and of the face probe, PMC FETCH / WRITE passes.
# usage: r3_final.sh TAG [skip-tests]
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/${1:-final}; mkdir -p $O
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu --maxfail=5 -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
  rc=$?
  grep -E "^FAILED|^ERROR" $O/gpu_tests.log | head -20; tail -2 $O/gpu_tests.log
  if [ $rc -ne 0 ]; then echo "tests rc $rc"; exit 1; fi
fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
cat $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_driver.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_bench -o run -- python3 $R/bench.py --no-cpu-baseline --no-extra > $O/prof_bench.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc_fetch -o run -- python3 $R/bench.py --steps 20 --warmup 1 --no-cpu-baseline --no-extra > $O/pmc_fetch.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmc_write -o run -- python3 $R/bench.py --steps 20 --warmup 1 --no-cpu-baseline --no-extra > $O/pmc_write.log 2>&1 || exit 1
# last: the face probe under rocprofv3 (its kernel stats are written; the process has segfaulted in
# its exit handlers after the profiler's finalisation on two boxes, so nothing runs after it)
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_face -o run -- python3 $R/scripts/face_probe.py 5 0 > $O/prof_face.log 2>&1
echo "face rocprof exit $?"
cd $R
for f in bench bench_driver; do grep '^{' $O/$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); e=d.get('extra',{}); print('$f', d['value'], d['ms_per_step'], d['roofline']['frac'], (d.get('roofline_hbm_smoother') or {}).get('frac'), (e.get('op1') or {}).get('vcycles_per_s'), (d.get('cpu_baseline') or {}).get('value'))"; done
echo "all ok"
