#!/bin/bash
# level-2 two-sweep passes at four waves per SIMD (no spill): op = 1 with PAMG_FACE_PP = 1 (level 1)
# vs 3 (levels 1 and 2), alternating, one box; the face tests first
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/r4i; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_face_operator.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do
  for pp in 1 3; do
    echo "== PAMG_FACE_PP=$pp rep $rep"
    PAMG_FACE_PP=$pp timeout -k 10 200 python scripts/face_probe.py 5 0 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
echo "all ok"
