#!/bin/bash
# round 6: the resident call at two workgroups per CU (dynamic LDS padding 40,960 B: 60 KB a workgroup) against
# three (no padding) -- the strong-scaling probe's per-rank shapes, alternating, one A/B build (PAMG_RESB_PAD)
set -o pipefail
O=gpurun_out/r6m; mkdir -p $O
for rep in 1 2; do
  for pad in 0 40960; do
    PAMG_LIB=scripts/ablibs/pad.so PAMG_RESB_PAD=$pad timeout -k 10 300 python -u scripts/strong_probe.py > $O/pad${pad}_$rep.txt 2>&1 || exit 1
  done
done
grep -H "N=" $O/pad*_*.txt | sed 's/(rank 0[^)]*)//'
