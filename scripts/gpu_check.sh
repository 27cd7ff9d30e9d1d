#!/bin/bash
# GPU-box check: smoke, GPU parity tests, bench, rocprofv3 kernel stats (csv).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
TAG=${1:-run}
echo "host: $(hostname) nproc=$(nproc)" > gpurun_out/env.txt
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 400 python bench.py --steps 50 --warmup 5 > gpurun_out/bench_$TAG.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$TAG -o run -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extra > $R/gpurun_out/prof_$TAG.log 2>&1
rc=$?
echo "exit $rc"
exit $rc
