#!/bin/bash
# round 5: the work before the warm-up at N = 1 and at an N = 8 rank's partition
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/r5q; mkdir -p $O
timeout -k 10 400 python scripts/prework_probe.py > $O/prework.txt 2>&1 || { tail $O/prework.txt; exit 1; }
grep -v amdgpu.ids $O/prework.txt
echo "all ok"
