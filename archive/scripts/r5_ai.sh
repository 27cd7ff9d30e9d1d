#!/bin/bash
# round 5 (session 2): the strong-scaling probe (detached partitions in the driver's call shape) with the resident call
# at four workgroups per CU (resb8) against three (base)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/r5ai; mkdir -p $O
for b in base resb8; do
  PAMG_LIB=$R/scripts/ablibs/$b.so timeout -k 10 400 python scripts/strong_probe.py > $O/strong_$b.txt 2>&1 || { tail $O/strong_$b.txt; exit 1; }
  echo "== $b"; grep -E "N=1|N=8" $O/strong_$b.txt
done
echo "all ok"
