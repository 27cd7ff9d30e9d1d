#!/bin/bash
# round 6: the ghost records -- bitwise against the gathers and the oracle (face tests), then timed against
# PAMG_FACE_GREC=0 in alternating processes
set -o pipefail
O=gpurun_out/r6k; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_face_operator.py > $O/face_tests.log 2>&1 || { tail -30 $O/face_tests.log; exit 1; }
tail -1 $O/face_tests.log
for rep in 1 2 3; do
  timeout -k 10 120 python -u scripts/face_probe.py 5 0,1 > $O/grec1_$rep.txt 2>&1 || exit 1
  PAMG_FACE_GREC=0 timeout -k 10 120 python -u scripts/face_probe.py 5 0,1 > $O/grec0_$rep.txt 2>&1 || exit 1
done
grep -H "V-cycles/s\|smooth" $O/grec*_*.txt
