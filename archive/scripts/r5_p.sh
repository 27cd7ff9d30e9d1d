#!/bin/bash
# round 5: the side measurements before the warm-up (default) against after the timed region (--extras-after),
# in the driver's shape (--steps 20 --warmup 5), alternating, without the CPU baseline
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/r5p; mkdir -p $O
for i in 1 2 3; do
  for m in first after; do
    f=""; [ $m = after ] && f="--extras-after"
    timeout -k 10 240 python bench.py --steps 20 --warmup 5 --no-cpu-baseline $f > $O/b_${m}_$i.json 2> $O/b_${m}_$i.err || { tail $O/b_${m}_$i.err; exit 1; }
    python - $O/b_${m}_$i.json $m $i <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], sys.argv[3], d["value"], d["ms_per_step"], d["roofline"]["frac"], d["roofline"]["ms_per_launch"], "op1", d["extra"]["op1"]["vcycles_per_s"], "tl", d["time_loop"]["vcycles_per_s"])
PY
  done
done
echo "all ok"
