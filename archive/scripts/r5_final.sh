#!/bin/bash
# Round-5 final evidence, in two calls (a call is limited to 20 minutes):
#   r5_final.sh TAG A   GPU tests, smoke, the bench (default and the driver's shape, with the CPU
#                       baseline), the strong-scaling probe, the coarsest-chain microbenchmark
#   r5_final.sh TAG B   rocprofv3 kernel stats of the bench (the driver's shape with its side measurements
#                       first, as bench.py runs it; the timed call's dispatch beside the bench line's events)
#                       and of the face probe, PMC FETCH / WRITE
#                       passes of the resident call and of the level-1 roofline sweeps
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/${1:-final}; mkdir -p $O
if [ "$2" = "A" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu --maxfail=5 -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
  rc=$?
  grep -E "^FAILED|^ERROR" $O/gpu_tests.log | head -20; tail -2 $O/gpu_tests.log
  if [ $rc -ne 0 ]; then echo "tests rc $rc"; exit 1; fi
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
  cat $O/smoke.log
  timeout -k 10 400 python bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.log 2>&1 || exit 1
  timeout -k 10 300 python scripts/strong_probe.py > $O/strong.txt 2>&1 || exit 1
  timeout -k 10 300 python scripts/xe_probe.py --calls 60 > $O/xe.txt 2>&1 || exit 1
  grep -E "median|charge|early" $O/xe.txt
  for f in bench bench_driver; do grep '^{' $O/$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); e=d.get('extra',{}); print('$f', d['value'], d['ms_per_step'], d['roofline']['frac'], (d.get('roofline_hbm_smoother') or {}).get('frac'), (e.get('op1') or {}).get('vcycles_per_s'), (e.get('op1_cycle1') or {}).get('vcycles_per_s'), (e.get('cycle1') or {}).get('vcycles_per_s'), (d.get('cpu_baseline') or {}).get('value'), ((d.get('cpu_baseline') or {}).get('all_cores') or {}).get('value'))"; done
fi
if [ "$2" = "B" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_bench -o run -- python3 $R/bench.py --no-cpu-baseline --no-extra > $O/prof_bench.log 2>&1 || exit 1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_bench_driver -o run -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/prof_bench_driver.log 2>&1 || exit 1
  python3 $R/scripts/trace_timed.py $O/prof_bench_driver "void pamg::(anonymous namespace)::k_vc_resb<5, 3" $O/prof_bench_driver.log > $O/prof_bench_driver_timed.txt || exit 1
  python3 $R/scripts/trace_timed.py $O/prof_bench "void pamg::(anonymous namespace)::k_vc_resb<5, 3" $O/prof_bench.log > $O/prof_bench_timed.txt || exit 1
  tail -2 $O/prof_bench_driver_timed.txt $O/prof_bench_timed.txt
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc_res_fetch -o run -- python3 $R/bench.py --steps 20 --warmup 1 --no-cpu-baseline --no-extra > $O/pmc_res_fetch.log 2>&1 || exit 1
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmc_res_write -o run -- python3 $R/bench.py --steps 20 --warmup 1 --no-cpu-baseline --no-extra > $O/pmc_res_write.log 2>&1 || exit 1
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc_sweep_fetch -o run -- python3 $R/scripts/sweep_prof.py 3 > $O/pmc_sweep_fetch.log 2>&1 || exit 1
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmc_sweep_write -o run -- python3 $R/scripts/sweep_prof.py 3 > $O/pmc_sweep_write.log 2>&1 || exit 1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_face -o run -- python3 $R/scripts/face_probe.py 5 0,1 > $O/prof_face.log 2>&1
  echo "face rocprof exit $?"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_xe -o run -- python3 $R/scripts/xe_probe.py --calls 20 > $O/prof_xe.log 2>&1
  echo "xe rocprof exit $?"
  cd $R
  timeout -k 10 400 python scripts/strong_probe.py > $O/strong_driver.txt 2>&1 || exit 1
  cat $O/strong_driver.txt
fi
if [ "$2" = "C" ]; then
  timeout -k 10 600 python scripts/cpu_baseline_probe.py > $O/cpu_probe.txt 2>&1 || { tail $O/cpu_probe.txt; exit 1; }
  cat $O/cpu_probe.txt
fi
echo "all ok"
