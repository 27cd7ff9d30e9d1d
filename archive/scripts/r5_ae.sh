#!/bin/bash
# round 5 (session 2): k_face_pp's start iterate and RHS into LDS by LDS-DMA (PAMG_FACE_PP_GLDS=1)
# where no correction is folded in: face tests, probe A/B against the previous build (scripts/ablibs/base.so); the
# matrix-free roofline sweep with x and b through LDS-DMA (PAMG_STENCIL_GLDS=1, default) against register loads (0)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/r5ae; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_face_operator.py > $O/t_face.log 2>&1 || { tail -30 $O/t_face.log; exit 1; }
tail -1 $O/t_face.log
for i in 1 2; do
  for b in base new; do
    if [ $b = base ]; then L=$R/scripts/ablibs/base.so; else L=; fi
    PAMG_LIB=$L timeout -k 10 200 python scripts/face_probe.py 5 0,1 > $O/probe_${b}_$i.txt 2>&1 || { tail $O/probe_${b}_$i.txt; exit 1; }
    echo "$b rep $i"; grep -E "V-cycles|smooth" $O/probe_${b}_$i.txt
  done
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_roofline_kernels.py > $O/t_roof.log 2>&1 || { tail -30 $O/t_roof.log; exit 1; }
tail -1 $O/t_roof.log
for i in 1 2 3; do
  for g in 0 1; do
    PAMG_STENCIL_GLDS=$g timeout -k 10 200 python scripts/asm_probe.py --reps 2 > $O/sten_${g}_$i.txt 2>&1 || { tail $O/sten_${g}_$i.txt; exit 1; }
    echo "stencil glds=$g"; grep assembled $O/sten_${g}_$i.txt
  done
done
echo "all ok"
