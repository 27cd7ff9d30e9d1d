#!/bin/bash
set -o pipefail
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  "tests/test_face_operator.py::test_face_operator_partitions_match_single_domain" \
  "tests/test_face_operator.py::test_agglomerated_coarsest_level_follows_state_set_between_calls" \
  tests/test_rccl_self.py > gpurun_out/r6_g.log 2>&1
