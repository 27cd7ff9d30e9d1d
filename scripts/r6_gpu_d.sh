#!/bin/bash
set -o pipefail
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread "tests/test_face_operator.py::test_agglomerated_coarsest_level_follows_state_set_between_calls" > gpurun_out/r6_d.log 2>&1 && \
bash scripts/final_evidence.sh r6b B && bash scripts/final_evidence.sh r6b C
