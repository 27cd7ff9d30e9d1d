#!/bin/bash
# round 5: k_sweep_assembled block layouts and plane gaps (A/B, interleaved), then its parity test
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/r5e; mkdir -p $O
: > $O/asm.txt
for round in 1 2; do
  for v in 01 11 12 14; do
    for pad in 0 4096; do
      PAMG_ASM_LAYOUT=$v PAMG_PITCH_PAD=$pad timeout -k 10 120 python scripts/asm_probe.py --reps 2 >> $O/asm.txt 2>&1 || { tail $O/asm.txt; exit 1; }
    done
  done
done
grep -v amdgpu.ids $O/asm.txt
for v in 01 11 12 14; do
  PAMG_ASM_LAYOUT=$v timeout -k 10 200 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests/test_roofline_kernels.py > $O/t_$v.log 2>&1 || { tail -20 $O/t_$v.log; exit 1; }
  echo "layout $v: $(tail -1 $O/t_$v.log)"
done
echo "all ok"
