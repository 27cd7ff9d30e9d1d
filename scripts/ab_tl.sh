#!/bin/bash
# A/B of library builds under scripts/ablibs on the reference-shaped time loop (scripts/time_loop_probe.py)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
: > gpurun_out/ab_tl.txt
for rep in 1 2 3; do
for f in scripts/ablibs/*.so; do
  r=$(PAMG_LIB=$PWD/$f timeout -k 10 100 python scripts/time_loop_probe.py 2>/dev/null) || exit 1
  echo "$(basename $f): $r" >> gpurun_out/ab_tl.txt
done
done
cat gpurun_out/ab_tl.txt
