#!/bin/bash
# round 5 (session 2): k_face_pp's ghost update from operands all gathered from memory, run before the tile's barrier
# (PAMG_FACE_PP_GHOST_EARLY=1): face tests, probe A/B against the previous build (scripts/ablibs/base.so)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/r5ab; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_face_operator.py > $O/t_face.log 2>&1 || { tail -30 $O/t_face.log; exit 1; }
tail -1 $O/t_face.log
for i in 1 2; do
  for b in base new; do
    if [ $b = base ]; then L=$R/scripts/ablibs/base.so; else L=; fi
    PAMG_LIB=$L timeout -k 10 200 python scripts/face_probe.py 5 0,1 > $O/probe_${b}_$i.txt 2>&1 || { tail $O/probe_${b}_$i.txt; exit 1; }
    echo "$b rep $i"; grep -E "V-cycles|smooth" $O/probe_${b}_$i.txt
  done
done
echo "all ok"
