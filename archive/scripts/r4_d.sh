#!/bin/bash
# Round-4 pass d: where the face sweeps' time goes -- kernel trace of the face probe (two-sweep passes),
# then SQ counter passes (issue, waits, LDS) on the same probe. Writes under gpurun_out/TAG.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r4d}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $O/counters_list.txt 2>&1
grep -o "SQ_[A-Z0-9_]*LDS[A-Z0-9_]*" $O/counters_list.txt | sort -u | head -20
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/scripts/face_probe.py 5 0 > $O/trace.log 2>&1 || { tail $O/trace.log; exit 1; }
head -20 $O/trace/run_kernel_stats.csv
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --kernel-trace --output-format csv -d $O/sq1 -o run -- python3 $R/scripts/face_probe.py 5 0 > $O/sq1.log 2>&1 || { tail $O/sq1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAVES --kernel-trace --output-format csv -d $O/sq2 -o run -- python3 $R/scripts/face_probe.py 5 0 > $O/sq2.log 2>&1 || { tail $O/sq2.log; exit 1; }
python3 $R/scripts/pmc_kernels.py k_face $O/sq1 $O/sq2 > $O/pmc_summary.txt
cat $O/pmc_summary.txt
