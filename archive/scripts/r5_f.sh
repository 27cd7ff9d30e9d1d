#!/bin/bash
# round 5: k_face_pp's first-round stagger (A/B, interleaved) on the face-operator cycle
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/r5f; mkdir -p $O
: > $O/stagger.txt
for round in 1 2; do
  for st in 0 400 800 1200; do
    echo "== stagger $st" >> $O/stagger.txt
    PAMG_FACE_PP_STAGGER=$st timeout -k 10 120 python scripts/face_probe.py 5 0 >> $O/stagger.txt 2>&1 || { tail $O/stagger.txt; exit 1; }
  done
done
grep -E "==|V-cycles|smooth" $O/stagger.txt
echo "all ok"
