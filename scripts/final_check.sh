#!/bin/bash
# Round evidence, final code: full_check.sh (smoke, GPU tests, bench, rocprof stats, PMC HBM
# passes), the driver's bench shape (--steps 20 --warmup 5) and one SQ/GRBM issue pass over
# the resident call. usage: final_check.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-final}
cd $R && mkdir -p gpurun_out
bash scripts/full_check.sh $TAG || exit 1
cd $R && timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_driver_$TAG.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && \
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d $R/gpurun_out/sq_$TAG -o run -- python3 $R/scripts/res_pmc.py > $R/gpurun_out/sq_$TAG.log 2>&1
rc=$?
echo "exit $rc"
exit $rc
