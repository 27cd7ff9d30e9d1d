#!/bin/bash
# round 5: k_face_pp with one snapshot image (three workgroups per CU): stamps, the face probe, the face tests
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/r5o; mkdir -p $O
timeout -k 10 300 python scripts/pp_stamps.py > $O/pp.txt 2>&1 || { tail $O/pp.txt; exit 1; }
cat $O/pp.txt
timeout -k 10 200 python scripts/face_probe.py 5 0,1 > $O/probe.txt 2>&1 || { tail $O/probe.txt; exit 1; }
grep -v amdgpu.ids $O/probe.txt
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_face_operator.py > $O/t_face.log 2>&1 || { tail -30 $O/t_face.log; exit 1; }
tail -1 $O/t_face.log
echo "all ok"
