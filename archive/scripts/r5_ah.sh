#!/bin/bash
# round 5 (session 2): the resident call at four workgroups per CU (PAMG_RESB_WAVES=8: 64 VGPRs, 68 B spilled per
# lane; 1,024 slots, so 8,192 tiles are 8 whole rounds) against three (the default build), in the driver's shape
# (bench.py --steps 20 --warmup 5) and the default, alternating processes
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/r5ah; mkdir -p $O
PAMG_LIB=$R/scripts/ablibs/resb8.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_contracted_oracle.py > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for i in 1 2 3; do
  for b in base resb8; do
    PAMG_LIB=$R/scripts/ablibs/$b.so timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/drv_${b}_$i.log 2>&1 || { tail $O/drv_${b}_$i.log; exit 1; }
    grep '^{' $O/drv_${b}_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$b driver', d['value'], d['roofline']['frac'])"
  done
done
for b in base resb8; do
  PAMG_LIB=$R/scripts/ablibs/$b.so timeout -k 10 200 python bench.py --no-cpu-baseline --no-extra > $O/def_${b}.log 2>&1 || { tail $O/def_${b}.log; exit 1; }
  grep '^{' $O/def_${b}.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$b default', d['value'], d['roofline']['frac'])"
done
echo "all ok"
