#!/bin/bash
# GPU-box A/B of the pipelined launch's dead-until-final stores: default (skipped) vs PAMG_PIPE_KEEP=7
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
for k in 0 7 0 7; do
  PAMG_PIPE_KEEP=$k timeout -k 10 120 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-extra > gpurun_out/keep_ab_$k.log 2>&1 || exit $?
  python -c "import json;d=json.loads(open('gpurun_out/keep_ab_$k.log').read().strip().splitlines()[-1]);print('keep=$k', d['value'], d['roofline']['achieved'], d['roofline']['frac'], d['roofline']['ms_per_launch'])" | tee -a gpurun_out/keep_ab.txt
done
