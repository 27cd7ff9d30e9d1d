#!/bin/bash
set -o pipefail
timeout -k 5 150 python -u scripts/agg_debug.py 900_ele.msh 2 2 2 0 > gpurun_out/aggdbg.txt 2>&1 && \
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  "tests/test_face_operator.py::test_face_operator_partitions_match_single_domain" \
  "tests/test_face_operator.py::test_face_chain_fallback_on_the_per_step_corrected_path" \
  "tests/test_face_operator.py::test_face_chain_not_coresident_falls_back_bitwise" tests/test_rccl_self.py > gpurun_out/r6_b.log 2>&1
