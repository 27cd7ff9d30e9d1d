#!/bin/bash
# round 6: XCD-grouped tiles of the face passes (default build) against the identity order (ablibs/facexcd0.so),
# alternating in separate processes; then the face tests on the default build
set -o pipefail
O=gpurun_out/r6e; mkdir -p $O
for rep in 1 2 3; do
  timeout -k 10 120 python -u scripts/face_probe.py 5 0,1 > $O/xcd1_$rep.txt 2>&1 || exit 1
  PAMG_LIB=scripts/ablibs/facexcd0.so timeout -k 10 120 python -u scripts/face_probe.py 5 0,1 > $O/xcd0_$rep.txt 2>&1 || exit 1
done
grep -H "V-cycles/s\|smooth" $O/xcd*_*.txt
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_face_operator.py > $O/face_tests.log 2>&1
