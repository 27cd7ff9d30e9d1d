#!/bin/bash
# HBM traffic of the hot kernels from rocprofv3 PMC counters, one counter group per pass
# (MI355X_MICROARCH.md: FETCH_SIZE and WRITE_SIZE cannot share a pass).
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-pmc}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/${TAG}_fetch -o run -- python3 $R/bench.py --steps 20 --warmup 1 --no-cpu-baseline --no-extra $BENCH_ARGS > $R/gpurun_out/${TAG}_fetch.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/${TAG}_write -o run -- python3 $R/bench.py --steps 20 --warmup 1 --no-cpu-baseline --no-extra $BENCH_ARGS > $R/gpurun_out/${TAG}_write.log 2>&1
echo "exit $?"
