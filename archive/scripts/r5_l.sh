#!/bin/bash
# round 5: the resident call's first-round stagger (A/B, interleaved)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/r5l; mkdir -p $O
for round in 1 2; do
  for cfg in "0 0" "100 0" "200 0" "100 1" "200 1"; do
    set -- $cfg
    PAMG_RES_STAGGER=$1 PAMG_RES_STAGGER_MODE=$2 timeout -k 10 120 python scripts/res_call_probe.py --tag "stagger=$1 mode=$2" >> $O/stagger.txt 2>&1 || { tail $O/stagger.txt; exit 1; }
  done
done
grep stagger $O/stagger.txt
echo "all ok"
