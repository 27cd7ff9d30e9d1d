#!/bin/bash
# A/B of library builds (scripts/ablibs) on the simulated N-rank partitions (tail_probe.py)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
: > gpurun_out/ab_strong.txt
for rep in 1 2; do
for f in scripts/ablibs/*.so; do
  echo "== $(basename $f)" >> gpurun_out/ab_strong.txt
  PAMG_LIB=$PWD/$f timeout -k 10 120 python scripts/tail_probe.py 2>/dev/null | grep -E "L=3 n_coarse=15" >> gpurun_out/ab_strong.txt || exit 1
done
done
cat gpurun_out/ab_strong.txt
