#!/bin/bash
R=$GRAFT_REPO_ROOT
cd $R; mkdir -p gpurun_out/ab
for v in base nohalo nouniform both; do
  case $v in base) E="";; nohalo) E="PAMG_DIAG_NOHALO=1";; nouniform) E="PAMG_DIAG_NOUNIFORM=1";; both) E="PAMG_DIAG_NOHALO=1 PAMG_DIAG_NOUNIFORM=1";; esac
  env $E timeout -k 10 200 python bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-extra > gpurun_out/ab/$v.log 2>&1 || exit 1
done
