#!/bin/bash
# A/B of the resident call's next-round cache warm-up (VArgs::pf_tiles, PAMG_RES_PF = cycle of the
# call in eighths, 0 off): the driver's shape and bench.py's default, alternating, one box
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/r4g; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_contracted_oracle.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do
  for pf in 0 4 7 2; do
    PAMG_RES_PF=$pf timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra > $O/drv_${pf}_$rep.log 2>&1 || exit 1
    echo "driver pf=$pf rep=$rep $(grep '^{' $O/drv_${pf}_$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['ms_per_launch'], d['roofline']['frac'])")"
  done
done
for pf in 0 4; do
  PAMG_RES_PF=$pf timeout -k 10 200 python bench.py --no-cpu-baseline --no-extra > $O/def_${pf}.log 2>&1 || exit 1
  echo "default pf=$pf $(grep '^{' $O/def_${pf}.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['ms_per_launch'], d['roofline']['frac'])")"
done
for pf in 0 4; do
  echo "== strong pf=$pf"
  PAMG_RES_PF=$pf timeout -k 10 400 python scripts/strong_probe.py 2>&1 | grep -v amdgpu.ids || exit 1
done
echo "all ok"
