#!/bin/bash
# round 5: early exchange at an N = 8 rank's shape (RCCL self-peer), in-packet events A/B
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/r5c; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu -s \
  tests/test_rccl_self.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
grep -E "passed|failed|early exchange" $O/tests.log | tail -4
timeout -k 10 200 python scripts/xe_probe.py > $O/xe_early.txt 2>&1 || { tail $O/xe_early.txt; exit 1; }
PAMG_EARLY_XC=0 timeout -k 10 200 python scripts/xe_probe.py > $O/xe_after.txt 2>&1 || { tail $O/xe_after.txt; exit 1; }
grep -v amdgpu.ids $O/xe_early.txt; grep -v amdgpu.ids $O/xe_after.txt
for k in 0 1 0 1; do
  PAMG_EVENTS_IN_PACKET=$k timeout -k 10 200 python scripts/shape_probe.py --reps 2 > $O/shape_pk$k.txt 2>&1 || { tail $O/shape_pk$k.txt; exit 1; }
  echo "in_packet=$k"; grep median $O/shape_pk$k.txt
done
echo "all ok"
