#!/bin/bash
# Fused face-operator sweep (k_face_sweep) vs the per-colour sequence (PAMG_FACE_FUSED=0) on
# bench.py's mesh, then the face-operator GPU tests. usage: face_check.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-face}
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_face_operator.py tests/test_corrected.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/face_tests_$TAG.log 2>&1 || { tail -30 gpurun_out/face_tests_$TAG.log; exit 1; }
tail -2 gpurun_out/face_tests_$TAG.log
for f in 0 1; do
  echo "== PAMG_FACE_FUSED=$f" >> gpurun_out/face_$TAG.txt
  PAMG_FACE_FUSED=$f timeout -k 10 120 python scripts/face_probe.py >> gpurun_out/face_$TAG.txt 2>&1 || exit 1
done
cat gpurun_out/face_$TAG.txt
