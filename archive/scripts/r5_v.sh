#!/bin/bash
# round 5: the reference face cycle's level-1 restrictor folded into the pass that computes its residual: face tests, probe A/B
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/r5v; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_face_operator.py > $O/t_face.log 2>&1 || { tail -30 $O/t_face.log; exit 1; }
tail -1 $O/t_face.log
for i in 1 2; do
  for rr in 0 1; do
    PAMG_FACE_RR=$rr timeout -k 10 200 python scripts/face_probe.py 5 0 > $O/probe_rr${rr}_$i.txt 2>&1 || { tail $O/probe_rr${rr}_$i.txt; exit 1; }
    echo "rr=$rr rep $i"; grep -v amdgpu.ids $O/probe_rr${rr}_$i.txt
  done
done
echo "all ok"
