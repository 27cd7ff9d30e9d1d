#!/bin/bash
# round 5 (session 2): k_face_pp with the gather entry's face pattern and the colour lists' fnb in tables of their own
# (one dependent load fewer at a pass's start): face tests, pass phase stamps (PAMG_STAMPS=1 build), probe A/B
# against the previous build (scripts/ablibs/base.so); the assembled roofline sweep on a resident grid with the next
# tile's loads in flight (PAMG_ASM_LAYOUT=21) against the tiled launch (12): its test, then interleaved probes
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/r5aa; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_face_operator.py > $O/t_face.log 2>&1 || { tail -30 $O/t_face.log; exit 1; }
tail -1 $O/t_face.log
timeout -k 10 300 python scripts/pp_stamps.py > $O/pp_stamps.txt 2>&1 || { tail $O/pp_stamps.txt; exit 1; }
grep -E "launches|phase" $O/pp_stamps.txt
for i in 1 2; do
  for b in base new; do
    if [ $b = base ]; then L=$R/scripts/ablibs/base.so; else L=; fi
    PAMG_LIB=$L timeout -k 10 200 python scripts/face_probe.py 5 0,1 > $O/probe_${b}_$i.txt 2>&1 || { tail $O/probe_${b}_$i.txt; exit 1; }
    echo "$b rep $i"; grep -E "V-cycles|smooth" $O/probe_${b}_$i.txt
  done
done
PAMG_ASM_LAYOUT=21 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_roofline_kernels.py > $O/t_roof.log 2>&1 || { tail -30 $O/t_roof.log; exit 1; }
tail -1 $O/t_roof.log
for i in 1 2 3; do
  for lay in 12 21; do
    PAMG_ASM_LAYOUT=$lay timeout -k 10 200 python scripts/asm_probe.py --reps 2 > $O/asm_${lay}_$i.txt 2>&1 || { tail $O/asm_${lay}_$i.txt; exit 1; }
    grep assembled $O/asm_${lay}_$i.txt
  done
done
echo "all ok"
