#!/bin/bash
# the per-wave chain with its snapshot offsets computed once per call (in-tree) vs per sweep
# (scripts/ablibs/libpamg_head.so, the previous HEAD): the face chain tests, then op = 1 alternating
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/r4n; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_face_operator.py -m gpu -x -q -k "per_wave or bitwise_the_oracle or two_sweep" --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do
  echo "== in-tree rep $rep"
  timeout -k 10 200 python scripts/face_probe.py 5 0 2>&1 | grep -v amdgpu.ids || exit 1
  echo "== previous HEAD rep $rep"
  PAMG_LIB=$R/scripts/ablibs/libpamg_head.so timeout -k 10 200 python scripts/face_probe.py 5 0 2>&1 | grep -v amdgpu.ids || exit 1
done
echo "all ok"
