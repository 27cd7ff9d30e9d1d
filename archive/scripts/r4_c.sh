#!/bin/bash
# Round-4 pass c: the face cycle's two-sweep passes (k_face_pp) -- their tests, then the face probe.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/${1:-r4c}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_face_operator.py -m gpu -k "two_sweep" -x -v --timeout 200 --timeout-method thread > $O/gpu_tests_pp.log 2>&1
rc=$?
grep -E "^FAILED|^ERROR|passed|failed" $O/gpu_tests_pp.log | tail -8
if [ $rc -ne 0 ]; then echo "pp tests rc $rc"; grep -B5 -A30 "Error\|assert" $O/gpu_tests_pp.log | head -60; exit 1; fi
timeout -k 10 200 python scripts/face_probe.py 5 0,1 > $O/face_probe.log 2>&1 || { tail -20 $O/face_probe.log; exit 1; }
cat $O/face_probe.log
PAMG_FACE_PP=0 timeout -k 10 200 python scripts/face_probe.py 5 0 > $O/face_probe_nopp.log 2>&1 || { tail -20 $O/face_probe_nopp.log; exit 1; }
cat $O/face_probe_nopp.log
timeout -k 10 900 python -u -m pytest tests/test_face_operator.py -m gpu -v --timeout 300 --timeout-method thread > $O/gpu_tests_face.log 2>&1
rc=$?
grep -E "^FAILED|^ERROR" $O/gpu_tests_face.log | head; tail -2 $O/gpu_tests_face.log
