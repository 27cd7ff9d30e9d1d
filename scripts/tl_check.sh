#!/bin/bash
# Resident time loop below n_split 5 / at L = 2: timing (one launch vs a launch per step) and
# the time-loop GPU tests. usage: tl_check.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-tl}
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "time_loop or contracted or multirank or schedule" > gpurun_out/tl_tests_$TAG.log 2>&1 || { tail -30 gpurun_out/tl_tests_$TAG.log; exit 1; }
tail -2 gpurun_out/tl_tests_$TAG.log
timeout -k 10 200 python scripts/tl_probe.py > gpurun_out/tl_$TAG.txt 2>&1 && \
PAMG_NO_RESIDENT_RUN=1 timeout -k 10 200 python scripts/tl_probe.py >> gpurun_out/tl_$TAG.txt 2>&1
rc=$?
cat gpurun_out/tl_$TAG.txt
exit $rc
