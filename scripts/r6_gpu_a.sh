#!/bin/bash
# round 6: RCCL missing-peer probe (modes 2, 1), then the agglomeration / RCCL / fallback tests
set -o pipefail
O=gpurun_out
( cd scripts/micro && timeout -k 5 30 ./nccl_init_probe 2 ) > $O/nip2.txt 2>&1; rc=$?; echo "rc=$rc" >> $O/nip2.txt
if [ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit $rc; fi
( cd scripts/micro && timeout -k 5 30 ./nccl_init_probe 1 ) > $O/nip1.txt 2>&1; rc=$?; echo "rc=$rc" >> $O/nip1.txt
if [ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit $rc; fi
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  "tests/test_face_operator.py::test_face_operator_partitions_match_single_domain" \
  "tests/test_face_operator.py::test_face_chain_fallback_on_the_per_step_corrected_path" \
  "tests/test_face_operator.py::test_face_chain_not_coresident_falls_back_bitwise" \
  tests/test_rccl_self.py -k "not missing_peer" > $O/r6_a.log 2>&1
