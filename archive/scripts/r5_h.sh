#!/bin/bash
# round 5: the chain's co-residency guard -- the CU-masked fallback test, the face tests, the guard's cost (A/B)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/r5h; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu \
  tests/test_face_operator.py -k "not_coresident" > $O/t_guard.log 2>&1 || { tail -40 $O/t_guard.log; exit 1; }
grep -E "passed|failed" $O/t_guard.log | tail -2
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_face_operator.py tests/test_rccl_self.py > $O/t_face.log 2>&1 || { tail -40 $O/t_face.log; exit 1; }
tail -2 $O/t_face.log
for k in 1 0 1 0; do
  echo "== PAMG_CHAIN_GUARD=$k" >> $O/probe.txt
  PAMG_CHAIN_GUARD=$k timeout -k 10 120 python scripts/face_probe.py 5 0,1 >> $O/probe.txt 2>&1 || { tail $O/probe.txt; exit 1; }
done
grep -E "==|V-cycles" $O/probe.txt
echo "all ok"
