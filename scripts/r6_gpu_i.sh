#!/bin/bash
# round 6: the face passes' tile loads issued before the ghost gathers (default build) against the old order
# (ablibs/oldorder.so), alternating processes; then the face tests on the default build
set -o pipefail
O=gpurun_out/r6i; mkdir -p $O
for rep in 1 2 3; do
  timeout -k 10 120 python -u scripts/face_probe.py 5 0,1 > $O/new_$rep.txt 2>&1 || exit 1
  PAMG_LIB=scripts/ablibs/oldorder.so timeout -k 10 120 python -u scripts/face_probe.py 5 0,1 > $O/old_$rep.txt 2>&1 || exit 1
done
grep -H "V-cycles/s\|smooth" $O/*_*.txt
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_face_operator.py > $O/face_tests.log 2>&1
