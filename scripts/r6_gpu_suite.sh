#!/bin/bash
# the whole GPU suite, one process (the round-end driver's form), then the driver's bench shape once more (the
# roofline.traffic from the committed PMC summary, whose digest now matches)
set -o pipefail
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r6_suite_final.log 2>&1 || { tail -30 gpurun_out/r6_suite_final.log; exit 1; }
tail -2 gpurun_out/r6_suite_final.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r6_bench_driver_final.log 2>&1 || { tail -20 gpurun_out/r6_bench_driver_final.log; exit 1; }
grep '^{' gpurun_out/r6_bench_driver_final.log | cut -c1-400
