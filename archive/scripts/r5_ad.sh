#!/bin/bash
# round 5 (session 2): the assembled roofline sweep with its block planes through LDS-DMA (PAMG_ASM_LAYOUT=31:
# global_load_lds_dwordx4 per plane piece; 41: x and b too) against the tiled register loads (12): tests, probes
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/r5ad; mkdir -p $O
for lay in 31 41; do PAMG_ASM_LAYOUT=$lay timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_roofline_kernels.py > $O/t_roof$lay.log 2>&1 || { tail -30 $O/t_roof$lay.log; exit 1; }; tail -1 $O/t_roof$lay.log; done

for i in 1 2 3; do
  for lay in 12 31 41; do
    PAMG_ASM_LAYOUT=$lay timeout -k 10 200 python scripts/asm_probe.py --reps 2 > $O/asm_${lay}_$i.txt 2>&1 || { tail $O/asm_${lay}_$i.txt; exit 1; }
    grep assembled $O/asm_${lay}_$i.txt
  done
done
echo "all ok"
