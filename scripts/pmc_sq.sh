#!/bin/bash
# SQ / TCC counter passes over a short fused bench run (one counter group per pass).
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-sq}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
run() {  # name counters...
  local name=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d $R/gpurun_out/${TAG}_$name -o run -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-extra $BENCH_ARGS > $R/gpurun_out/${TAG}_$name.log 2>&1
}
timeout -s KILL 60 rocprofv3 -L > $R/gpurun_out/counters_list.txt 2>&1
run fetch FETCH_SIZE && run write WRITE_SIZE && \
run sq1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY && \
run sq2 SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT
echo "exit $?"
