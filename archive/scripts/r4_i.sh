#!/bin/bash
# level-2 two-sweep passes at four waves per SIMD (no spill; scripts/ablibs/libpamg_pp256.so, built from
# the in-tree sources with that launch bound): the face tests on it, then op = 1 with PAMG_FACE_PP = 1
# (level 1) vs 3 (levels 1 and 2), in-tree vs the variant, alternating, one box
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/r4i; mkdir -p $O
AB=$R/scripts/ablibs/libpamg_pp256.so
PAMG_LIB=$AB timeout -k 10 400 python -u -m pytest tests/test_face_operator.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do
  echo "== in-tree PAMG_FACE_PP=1 rep $rep"
  PAMG_FACE_PP=1 timeout -k 10 200 python scripts/face_probe.py 5 0 2>&1 | grep -v amdgpu.ids || exit 1
  echo "== in-tree PAMG_FACE_PP=3 rep $rep"
  PAMG_FACE_PP=3 timeout -k 10 200 python scripts/face_probe.py 5 0 2>&1 | grep -v amdgpu.ids || exit 1
  echo "== pp256 PAMG_FACE_PP=3 rep $rep"
  PAMG_LIB=$AB PAMG_FACE_PP=3 timeout -k 10 200 python scripts/face_probe.py 5 0 2>&1 | grep -v amdgpu.ids || exit 1
done
echo "all ok"
