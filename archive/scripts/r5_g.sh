#!/bin/bash
# round 5: the corrected face cycle in two-sweep passes -- its tests, then the probe (A/B with PAMG_FACE_CORR_PP=0)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/r5g; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_face_operator.py -k "corrected_cycle_passes or bitwise_the_oracle" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -3
for k in 1 0 1 0; do
  echo "== PAMG_FACE_CORR_PP=$k" >> $O/probe.txt
  PAMG_FACE_CORR_PP=$k timeout -k 10 120 python scripts/face_probe.py 5 1 >> $O/probe.txt 2>&1 || { tail $O/probe.txt; exit 1; }
done
grep -v amdgpu.ids $O/probe.txt
echo "all ok"
