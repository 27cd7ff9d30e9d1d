#!/bin/bash
# round 5 checkpoint: the whole GPU suite, the exchange probe with the deferred join, the driver-shape bench
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/r5j; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 200 python scripts/xe_probe.py --calls 60 > $O/xe.txt 2>&1 || { tail $O/xe.txt; exit 1; }
grep -E "median|charge|early" $O/xe.txt
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench.json'));e=d['extra'];print(d['value'],d['roofline']['frac'],d['roofline_hbm_smoother']['frac'],e['op1']['vcycles_per_s'],e['op1_cycle1']['vcycles_per_s'],e['cycle1']['vcycles_per_s'])"
echo "all ok"
