#!/bin/bash
# round 6: the level-2 folded pass instance (cycle 1) at six waves per SIMD (PAMG_FACE_PP_WAVES256=6: 79 VGPRs, 12 B
# spilled) against five (81 VGPRs), op = 1 cycle 1 alternating pairs
set -o pipefail
O=gpurun_out/r6t; mkdir -p $O
for rep in 1 2 3 4; do
  timeout -k 10 120 python -u scripts/face_probe.py 5 1 > $O/base_$rep.txt 2>&1 || exit 1
  PAMG_LIB=scripts/ablibs/w6.so timeout -k 10 120 python -u scripts/face_probe.py 5 1 > $O/w6_$rep.txt 2>&1 || exit 1
done
grep -H "V-cycles/s\|smooth " $O/base_*.txt $O/w6_*.txt
