#!/bin/bash
# the driver shape's clock ramp (scripts/ramp_probe.py) and the PMC passes of the pipelined launch
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/r4h; mkdir -p $O
timeout -k 10 200 python scripts/ramp_probe.py > $O/ramp.txt 2>&1 || { tail $O/ramp.txt; exit 1; }
grep -v amdgpu.ids $O/ramp.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc_pipe_fetch -o run -- python3 $R/scripts/pipe_prof.py 20 > $O/pmc_pipe_fetch.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmc_pipe_write -o run -- python3 $R/scripts/pipe_prof.py 20 > $O/pmc_pipe_write.log 2>&1 || exit 1
echo "all ok"
