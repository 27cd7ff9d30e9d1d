#!/bin/bash
# round 5 (session 3): the level-2 two-sweep passes (k_face_pp<256, 192>, no folded interpolation) at eight
# waves per SIMD (63 VGPRs, SGPR spills into VGPR lanes, no scratch) instead of four (80 VGPRs, six): face tests
# on that build (bitwise), probe A/B against this build (scripts/ablibs/w8.so: PAMG_FACE_PP_WAVES256_PLAIN=8)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/r5aq; mkdir -p $O
PAMG_LIB=$R/scripts/ablibs/w8.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_face_operator.py > $O/t_face_w8.log 2>&1 || { tail -30 $O/t_face_w8.log; exit 1; }
tail -1 $O/t_face_w8.log
run() {   # tag lib
  if [ $2 = w8 ]; then L=$R/scripts/ablibs/w8.so; else L=; fi
  PAMG_LIB=$L timeout -k 10 200 python scripts/face_probe.py 5 0,1 > $O/probe_$1.txt 2>&1 || { tail $O/probe_$1.txt; exit 1; }
  echo "$1"; grep -v amdgpu.ids $O/probe_$1.txt
}
for i in 1 2; do
  run w4_$i w4 || exit 1
  run w8_$i w8 || exit 1
done
echo "all ok"
