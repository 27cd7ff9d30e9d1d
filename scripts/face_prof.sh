#!/bin/bash
# The face-coupled operator (op = 1) on bench.py's mesh: event-timed probe, rocprofv3 kernel stats,
# PMC bytes and SQ counters of its kernels (one counter group per pass). usage: face_prof.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-face}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R && timeout -k 10 300 python scripts/face_probe.py > $O/face_probe.txt 2>&1 || { tail $O/face_probe.txt; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/scripts/face_probe.py > $O/prof.log 2>&1 || exit 1
run() {  # name counters...
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d $O/pmc_$name -o run -- python3 $R/scripts/face_probe.py 5 0 > $O/pmc_$name.log 2>&1
}
run fetch FETCH_SIZE && run write WRITE_SIZE && \
run sq1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY && \
run sq2 SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT
echo "exit $?"
