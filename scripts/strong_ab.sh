#!/bin/bash
# Simulated per-rank strong scaling (scripts/strong_probe.py) of the in-tree library and of
# the A/B builds under scripts/ablibs. usage: strong_ab.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-strong}
cd $R && mkdir -p gpurun_out
echo "== in-tree" >> gpurun_out/strong_$TAG.txt
timeout -k 10 200 python scripts/strong_probe.py >> gpurun_out/strong_$TAG.txt 2>&1 || exit 1
for f in scripts/ablibs/*.so; do
  echo "== $(basename $f)" >> gpurun_out/strong_$TAG.txt
  PAMG_RES_PAIR=0 PAMG_LIB=$PWD/$f timeout -k 10 200 python scripts/strong_probe.py >> gpurun_out/strong_$TAG.txt 2>&1 || exit 1
done
cat gpurun_out/strong_$TAG.txt
