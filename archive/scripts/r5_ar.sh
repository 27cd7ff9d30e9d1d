#!/bin/bash
# round 5 (session 3): the coarsest level's two smoother calls of a cycle that is not the call's last as one call
# (PAMG_FACE_COARSE_MERGE, default 1): the face suite (bitwise), and face_probe.py 5 0,1 with the merge and without
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/r5ar; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_face_operator.py > $O/t_face.log 2>&1 || { tail -30 $O/t_face.log; exit 1; }
tail -1 $O/t_face.log
run() {   # tag merge
  PAMG_FACE_COARSE_MERGE=$2 timeout -k 10 200 python scripts/face_probe.py 5 0,1 > $O/probe_$1.txt 2>&1 || { tail $O/probe_$1.txt; exit 1; }
  echo "$1"; grep -v amdgpu.ids $O/probe_$1.txt
}
for i in 1 2; do
  run two_$i 0 || exit 1
  run merged_$i 1 || exit 1
done
echo "all ok"
