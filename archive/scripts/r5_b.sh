#!/bin/bash
# round 5: the early per-call exchange (local group + RCCL self-peer), the in-packet timing events, the bench shape
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/r5b; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu -s \
  tests/test_rccl_self.py tests/test_multirank.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
grep -E "passed|failed|early exchange" $O/tests.log | tail -8
timeout -k 10 200 python scripts/shape_probe.py --reps 3 > $O/shape.txt 2>&1 || { tail $O/shape.txt; exit 1; }
grep median $O/shape.txt
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench.json'));print(d['value'],d['roofline']['frac'],d['roofline_hbm_smoother']['frac'],d['extra']['op1']['vcycles_per_s'])"
echo "all ok"
