#!/bin/bash
# the per-wave chain with its flag after the down pass (PAMG_CHAIN_EARLY=4: the drain under the down pass)
# vs before it (default): the face tests under 4 first (per-wave vs workgroup chain, oracle cases), then
# op = 1 alternating, one box
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/r4m; mkdir -p $O
PAMG_CHAIN_EARLY=4 timeout -k 10 500 python -u -m pytest tests/test_face_operator.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { grep -E "FAIL|Error" $O/tests.log | head -20; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u -m pytest tests/test_face_operator.py -m gpu -x -q -k "per_wave or bitwise_the_oracle" --timeout 300 --timeout-method thread > $O/tests3.log 2>&1 || { tail -30 $O/tests3.log; exit 1; }
tail -1 $O/tests3.log
for rep in 1 2; do
  echo "== early 4 rep $rep"
  PAMG_CHAIN_EARLY=4 timeout -k 10 200 python scripts/face_probe.py 5 0 2>&1 | grep -v amdgpu.ids || exit 1
  echo "== early 3 (default) rep $rep"
  timeout -k 10 200 python scripts/face_probe.py 5 0 2>&1 | grep -v amdgpu.ids || exit 1
done
echo "all ok"
