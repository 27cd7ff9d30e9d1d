#!/bin/bash
# Evidence for DESIGN.md / profiles (one GPU box; a call is limited to 20 minutes):
#   final_evidence.sh TAG A   smoke, the bench (default and the driver's shape, with the CPU baseline), the
#                             strong-scaling probe, the face-operator partition probe
#   final_evidence.sh TAG B   rocprofv3 kernel stats of the bench in the driver's shape (the timed call's dispatch
#                             beside the bench line's events) and of the face probe; PMC FETCH / WRITE passes of
#                             the resident call and of the level-1 roofline sweeps (separate --pmc runs)
#   final_evidence.sh TAG C   SQ issue / wait counters and HBM bytes of the op = 1 passes (face probe, cycle 0)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/${1:-final}; mkdir -p $O
if [ "$2" = "A" ]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
  cat $O/smoke.log
  timeout -k 10 500 python bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
  timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.log 2>&1 || { tail -20 $O/bench_driver.log; exit 1; }
  for f in bench bench_driver; do grep '^{' $O/$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); e=d.get('extra',{}); print('$f', d['value'], d['ms_per_step'], d['roofline']['frac'], (d.get('roofline_hbm_smoother') or {}).get('frac'), (e.get('op1') or {}).get('vcycles_per_s'), (e.get('op1_cycle1') or {}).get('vcycles_per_s'), (e.get('cycle1') or {}).get('vcycles_per_s'), (d.get('cpu_baseline') or {}).get('value'), ((d.get('cpu_baseline') or {}).get('all_cores') or {}).get('value'))"; done
  timeout -k 10 400 python scripts/strong_probe.py > $O/strong.txt 2>&1 || exit 1
  timeout -k 10 300 python -u scripts/face_strong_probe.py 5 10 1 > $O/face_partitions.txt 2>&1 || exit 1
  # the multi-rank orchestration of bench.py (rendezvous, barrier before the communicator, MAX over ranks) on one
  # GPU: two detached ranks (RCCL refuses two ranks on one GPU; the exchange itself is tests/test_rccl_self.py's)
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
      --master-port 29531 bench.py --gpus 2 --steps 20 --warmup 5 --comm detached > $O/bench_2ranks_detached.log 2>&1 || \
      { tail -20 $O/bench_2ranks_detached.log; exit 1; }
  grep '^{' $O/bench_2ranks_detached.log | cut -c1-300
fi
if [ "$2" = "B" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_bench_driver -o run -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/prof_bench_driver.log 2>&1 || exit 1
  python3 $R/scripts/trace_timed.py $O/prof_bench_driver "void pamg::(anonymous namespace)::k_vc_resb<5, 3" $O/prof_bench_driver.log > $O/prof_bench_driver_timed.txt || exit 1
  tail -2 $O/prof_bench_driver_timed.txt
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc_res_fetch -o run -- python3 $R/bench.py --steps 20 --warmup 1 --no-cpu-baseline --no-extra > $O/pmc_res_fetch.log 2>&1 || exit 1
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmc_res_write -o run -- python3 $R/bench.py --steps 20 --warmup 1 --no-cpu-baseline --no-extra > $O/pmc_res_write.log 2>&1 || exit 1
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc_sweep_fetch -o run -- python3 $R/scripts/sweep_prof.py 3 > $O/pmc_sweep_fetch.log 2>&1 || exit 1
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmc_sweep_write -o run -- python3 $R/scripts/sweep_prof.py 3 > $O/pmc_sweep_write.log 2>&1 || exit 1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_face -o run -- python3 $R/scripts/face_probe.py 5 0,1 > $O/prof_face.log 2>&1
  echo "face rocprof exit $?"
fi
if [ "$2" = "C" ]; then
  # the op = 1 level-1 two-sweep pass's issue and wait counters (separate --pmc runs, one SQ group each)
  cd /tmp && export TMPDIR=/tmp
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY --kernel-trace --output-format csv -d $O/sq_face1 -o run -- python3 $R/scripts/face_probe.py 5 0 > $O/sq_face1.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d $O/sq_face2 -o run -- python3 $R/scripts/face_probe.py 5 0 > $O/sq_face2.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc_face_fetch -o run -- python3 $R/scripts/face_probe.py 5 0 > $O/pmc_face_fetch.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmc_face_write -o run -- python3 $R/scripts/face_probe.py 5 0 > $O/pmc_face_write.log 2>&1 || exit 1
fi
echo "all ok"
