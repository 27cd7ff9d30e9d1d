#!/bin/bash
# the per-wave chain (k_face_chain_pw): the face tests (incl. per-wave vs workgroup chain bitwise), then
# op = 1 with PAMG_CHAIN_PW = 1 vs 0, alternating, one box
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/r4j; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_face_operator.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { grep -E "FAIL|Error|error" $O/tests.log | head -20; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do
  for pw in 1 0; do
    echo "== PAMG_CHAIN_PW=$pw rep $rep"
    PAMG_CHAIN_PW=$pw timeout -k 10 200 python scripts/face_probe.py 5 0 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
echo "all ok"
