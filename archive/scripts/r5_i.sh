#!/bin/bash
# round 5: what is left of a call's exchange cost at the N = 8 shape: the join barrier (PAMG_XE_NOJOIN=1, timing only)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/r5i; mkdir -p $O
for k in 0 1 0 1; do
  echo "== PAMG_XE_NOJOIN=$k" >> $O/xe.txt
  PAMG_XE_NOJOIN=$k timeout -k 10 200 python scripts/xe_probe.py --calls 60 >> $O/xe.txt 2>&1 || { tail $O/xe.txt; exit 1; }
done
grep -E "==|median|charge|early" $O/xe.txt
echo "all ok"
