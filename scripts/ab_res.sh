#!/bin/bash
# A/B of resident-kernel library builds (scripts/ablibs/*.so via PAMG_LIB), interleaved on one
# box: res_probe.py (bitwise check, calls of 200 / 20 cycles, the time loop); then the GPU tests
# of the fused / resident forms on the in-tree library. usage: ab_res.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-ab}
cd $R && mkdir -p gpurun_out
for rep in 1 2; do
  for f in scripts/ablibs/*.so; do
    echo "== $(basename $f) rep $rep" >> gpurun_out/abres_$TAG.txt
    PAMG_RES_PAIR=0 PAMG_LIB=$PWD/$f timeout -k 10 120 python scripts/res_probe.py >> gpurun_out/abres_$TAG.txt 2>&1 || exit 1
  done
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/abres_tests_$TAG.log 2>&1
rc=$?
tail -3 gpurun_out/abres_tests_$TAG.log
exit $rc
