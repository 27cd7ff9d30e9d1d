#!/bin/bash
# round 6: the coarser levels' restrictor fold, more alternating A/B pairs (op = 1, cycle 0, face_probe.py 5 0)
set -o pipefail
O=gpurun_out/r6r; mkdir -p $O
for rep in 1 2 3 4 5 6; do
  PAMG_LIB=scripts/ablibs/base.so timeout -k 10 120 python -u scripts/face_probe.py 5 0 > $O/base_$rep.txt 2>&1 || exit 1
  timeout -k 10 120 python -u scripts/face_probe.py 5 0 > $O/fold_$rep.txt 2>&1 || exit 1
done
grep -H "V-cycles/s" $O/base_*.txt $O/fold_*.txt
