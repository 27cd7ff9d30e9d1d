#!/bin/bash
# round 6: edge cases -- the one-element mesh (op = 0 and 1), zero-cycle / zero-step calls
set -o pipefail
O=gpurun_out/r6o; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_edge_cases.py -x -v --timeout 120 --timeout-method thread \
  -m gpu > $O/tests.txt 2>&1 || { tail -60 $O/tests.txt; exit 1; }
tail -3 $O/tests.txt
