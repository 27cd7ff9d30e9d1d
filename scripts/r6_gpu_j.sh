#!/bin/bash
# round 6: which part of the face passes' ghost update costs (timing diagnostics, wrong results): no gathers at all,
# the operands loaded but the update not computed, the gather entry read but its operands not loaded
set -o pipefail
O=gpurun_out/r6j; mkdir -p $O
for rep in 1 2; do
  timeout -k 10 120 python -u scripts/face_probe.py 5 0 > $O/base_$rep.txt 2>&1 || exit 1
  for v in nogather noghostcalc noghostloads; do
    PAMG_LIB=scripts/ablibs/$v.so timeout -k 10 120 python -u scripts/face_probe.py 5 0 > $O/${v}_$rep.txt 2>&1 || exit 1
  done
done
grep -H "V-cycles/s\|smooth" $O/*_*.txt
