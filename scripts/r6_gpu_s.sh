#!/bin/bash
# round 6: PMC FETCH / WRITE passes of the one-launch-per-cycle form's pipelined launch at the final sources
# (profiles/pmc_vcycle_pipe.json, bench.py's extra.one_launch_per_cycle traffic)
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6s; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc_pipe_fetch -o run -- python3 $R/scripts/pipe_prof.py 20 > $O/pmc_pipe_fetch.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmc_pipe_write -o run -- python3 $R/scripts/pipe_prof.py 20 > $O/pmc_pipe_write.log 2>&1 || exit 1
echo ok
