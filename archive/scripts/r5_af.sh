#!/bin/bash
# round 5 (session 2): k_face_pp's LDS-DMA loads in the folded passes too (the corrected cycle's interpolation added
# to X in place): face tests, probes (compare r05_ae's 674-676 for the corrected cycle)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/r5af; mkdir -p $O
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
