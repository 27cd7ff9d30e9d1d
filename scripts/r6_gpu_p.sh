#!/bin/bash
# round 6: edge cases incl. ranks that own no un_ele
set -o pipefail
O=gpurun_out/r6p; mkdir -p $O
PAMG_COMM_TIMEOUT_S=20 timeout -k 10 600 python -u -m pytest tests/test_edge_cases.py -x -v --timeout 120 --timeout-method thread \
  -m gpu > $O/tests.txt 2>&1 || { tail -60 $O/tests.txt; exit 1; }
tail -3 $O/tests.txt
