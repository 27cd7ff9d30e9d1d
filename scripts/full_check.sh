#!/bin/bash
# Round evidence: smoke, all GPU tests, bench, rocprofv3 kernel stats, PMC HBM traffic passes.
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-run}
cd $R && mkdir -p gpurun_out
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 400 python bench.py > gpurun_out/bench_$TAG.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$TAG -o run -- python3 $R/bench.py --no-cpu-baseline --no-extra > $R/gpurun_out/prof_$TAG.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/pmc_${TAG}_fetch -o run -- python3 $R/bench.py --steps 20 --warmup 1 --no-cpu-baseline --no-extra > $R/gpurun_out/pmc_${TAG}_fetch.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/pmc_${TAG}_write -o run -- python3 $R/bench.py --steps 20 --warmup 1 --no-cpu-baseline --no-extra > $R/gpurun_out/pmc_${TAG}_write.log 2>&1
rc=$?
echo "exit $rc"
exit $rc
