#!/bin/bash
# A/B of library builds under scripts/ablibs (PAMG_LIB), interleaved, same box.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
: > gpurun_out/ab2.txt
for rep in 1 2 3; do
for f in scripts/ablibs/*.so; do
  r=$(PAMG_LIB=$PWD/$f timeout -k 10 60 python scripts/ab_probe.py ${AB_CASES:-5,3,3,1 5,3,1,1} 2>/dev/null) || exit 1
  echo "$(basename $f): $r" >> gpurun_out/ab2.txt
done
done
cat gpurun_out/ab2.txt
