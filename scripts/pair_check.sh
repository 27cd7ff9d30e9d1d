#!/bin/bash
# Two-tile resident kernel: A/B against the one-tile balanced kernel (PAMG_RES_PAIR), then the
# resident-form GPU tests. usage: pair_check.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-pair}
cd $R && mkdir -p gpurun_out
for rep in 1 2; do
  for p in 0 1; do
    echo "== PAMG_RES_PAIR=$p rep $rep" >> gpurun_out/pair_$TAG.txt
    PAMG_RES_PAIR=$p timeout -k 10 120 python scripts/res_probe.py >> gpurun_out/pair_$TAG.txt 2>&1 || exit 1
  done
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "fused or resident or schedule or time_loop or partition or contracted or multirank" > gpurun_out/pair_tests_$TAG.log 2>&1
rc=$?
tail -3 gpurun_out/pair_tests_$TAG.log
exit $rc
