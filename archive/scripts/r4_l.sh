#!/bin/bash
# at HEAD: the face probe under rocprofv3 (kernel stats of the final face kernels), the corrected cycle on
# the face operator (op = 1, cycle = 1) for reference
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/r4l; mkdir -p $O
timeout -k 10 200 python scripts/face_probe.py 5 1 > $O/face_cycle1.txt 2>&1 || { tail $O/face_cycle1.txt; exit 1; }
grep -v amdgpu.ids $O/face_cycle1.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_face -o run -- python3 $R/scripts/face_probe.py 5 0 > $O/prof_face.log 2>&1
echo "face rocprof exit $?"
head -8 $O/prof_face/run_kernel_stats.csv | cut -c1-160
