#!/bin/bash
# round 6: the face operator's partitions with four levels (the coarsest agglomerated below two partitioned ones)
set -o pipefail
O=gpurun_out/r6n; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_face_operator.py -x -v --timeout 200 --timeout-method thread \
  -k "partitions_match" -m gpu > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
tail -3 $O/tests.txt
