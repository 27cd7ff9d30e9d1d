#!/bin/bash
# round 5: the folded first pass (interpolation) at six waves per SIMD (28-32 B spilled) or five (no spill, two workgroups per CU)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/r5t; mkdir -p $O
for i in 1 2; do
  timeout -k 10 200 python scripts/face_probe.py 5 1 > $O/probe_w6_$i.txt 2>&1 || { tail $O/probe_w6_$i.txt; exit 1; }
  echo "waves 6 rep $i"; grep -v amdgpu.ids $O/probe_w6_$i.txt
  PAMG_LIB=$R/scripts/ablibs/fw5.so timeout -k 10 200 python scripts/face_probe.py 5 1 > $O/probe_w5_$i.txt 2>&1 || { tail $O/probe_w5_$i.txt; exit 1; }
  echo "waves 5 rep $i"; grep -v amdgpu.ids $O/probe_w5_$i.txt
done
echo "all ok"
