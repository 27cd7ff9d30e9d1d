#!/bin/bash
# GPU parity tests of the fused V-cycle (both schedules), then the concurrency probe.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "fused or contracted or pipelined" --timeout 120 --timeout-method thread > gpurun_out/conc_tests.log 2>&1 && \
timeout -k 10 180 python -u scripts/conc_probe.py > gpurun_out/conc_probe.txt 2>&1
rc=$?
echo "exit $rc"
exit $rc
