#!/bin/bash
# A/B of the face operator kernel forms (env switches) on bench.py mesh (face_probe, cycle 0), interleaved twice
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/${1:-faceab}; mkdir -p $O
for rep in 1 2; do
  for v in "PAMG_FACE_CMP=1 PAMG_FACE_CHAIN=1" "PAMG_FACE_CMP=0 PAMG_FACE_CHAIN=1" "PAMG_FACE_CMP=1 PAMG_FACE_CHAIN=0" "PAMG_FACE_CMP=0 PAMG_FACE_CHAIN=0"; do
    echo "== $v rep $rep" >> $O/ab.txt
    env $v timeout -k 10 200 python scripts/face_probe.py 5 0 >> $O/ab.txt 2>&1 || exit 1
  done
done
grep -E "==|V-cycles|smooth" $O/ab.txt
