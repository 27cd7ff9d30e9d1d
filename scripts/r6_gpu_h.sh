#!/bin/bash
# round 6: the op = 1 passes without their gathers (timing diagnostic, wrong results) -- the upper bound of any
# change to the ghost updates' operand loads
set -o pipefail
O=gpurun_out/r6h; mkdir -p $O
for rep in 1 2; do
  timeout -k 10 120 python -u scripts/face_probe.py 5 0 > $O/base_$rep.txt 2>&1 || exit 1
  PAMG_LIB=scripts/ablibs/nogather.so timeout -k 10 120 python -u scripts/face_probe.py 5 0 > $O/nogather_$rep.txt 2>&1 || exit 1
done
grep -H "V-cycles/s\|smooth" $O/*.txt
