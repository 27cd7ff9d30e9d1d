#!/bin/bash
# Quick GPU iteration: GPU parity tests, fused V-cycle timing variants, phase stamps.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 120 python scripts/vc_probe.py ${VC_CASES:-5,3,4,15 5,3,4,1 3,3,4,15} > gpurun_out/vc_probe.txt 2>&1
rc=$?
echo "exit $rc"
exit $rc
