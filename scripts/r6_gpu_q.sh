#!/bin/bash
# round 6: the face cycle's coarser streaming levels fold their restrictor into the pass that computes the residual
# (level 2 -> level 3's second RHS buffer) -- the face tests bitwise, then A/B V-cycles/s against the build before it
set -o pipefail
O=gpurun_out/r6q; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_face_operator.py tests/test_edge_cases.py -x -v --timeout 200 \
  --timeout-method thread -m gpu > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
tail -3 $O/tests.txt
for rep in 1 2 3; do
  PAMG_LIB=scripts/ablibs/base.so timeout -k 10 120 python -u scripts/face_probe.py 5 > $O/base_$rep.txt 2>&1 || exit 1
  timeout -k 10 120 python -u scripts/face_probe.py 5 > $O/fold_$rep.txt 2>&1 || exit 1
done
grep -H "V-cycles/s\|smooth \|restrict" $O/base_*.txt $O/fold_*.txt
