#!/bin/bash
# Round-4 pass e: A/B of the two-sweep face pass variants (RHS in LDS or registers, waves per SIMD) and of
# the corrected resident call's occupancy, on one box. scripts/ablibs/*.so via PAMG_LIB.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/${1:-r4e}; mkdir -p $O
for rep in 1 2; do
  for lib in ppA ppB ppC; do
    echo "== $lib rep $rep"
    PAMG_LIB=$R/scripts/ablibs/$lib.so timeout -k 10 120 python scripts/face_probe.py 5 0 2>&1 | grep -v amdgpu.ids || exit 1
  done
  echo "== one-sweep launches rep $rep"
  PAMG_FACE_PP=0 timeout -k 10 120 python scripts/face_probe.py 5 0 2>&1 | grep -v amdgpu.ids || exit 1
  echo "== ppA with level 2 streaming too rep $rep"
  PAMG_FACE_PP=3 PAMG_LIB=$R/scripts/ablibs/ppA.so timeout -k 10 120 python scripts/face_probe.py 5 0 2>&1 | grep -v amdgpu.ids || exit 1
done > $O/face_ab.log
cat $O/face_ab.log | grep -E "==|V-cycles"
for rep in 1 2; do
  for lib in default corrW8; do
    echo "== corrected $lib rep $rep"
    if [ $lib = default ]; then L=; else L=$R/scripts/ablibs/$lib.so; fi
    PAMG_LIB=$L timeout -k 10 120 python scripts/corr_probe.py 5 3 200 2>&1 | grep -v amdgpu.ids || exit 1
  done
done > $O/corr_ab.log
cat $O/corr_ab.log
timeout -k 10 300 python scripts/face_strong_probe.py 5 10 > $O/face_strong.log 2>&1 || { tail -5 $O/face_strong.log; exit 1; }
grep -v amdgpu.ids $O/face_strong.log
