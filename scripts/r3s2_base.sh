#!/bin/bash
# Session-2 baseline pass on the rebuilt tree: all GPU tests, the bench (no CPU baseline), the
# face-operator probe with the chain's phase stamps. usage: r3s2_base.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/${1:-base}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu --maxfail=10 -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?
grep -E "^FAILED|^ERROR" $O/gpu_tests.log | head -20; tail -2 $O/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit 1; fi
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
timeout -k 10 300 python scripts/face_probe.py 5 0 > $O/face_probe.txt 2>&1 || { tail $O/face_probe.txt; exit 1; }
cat $O/face_probe.txt
rm -f $O/chain_stamps.bin
PAMG_CHAIN_STAMPS=$O/chain_stamps.bin timeout -k 10 300 python scripts/face_probe.py 5 0 > $O/face_probe_stamps.txt 2>&1 || exit 1
python3 scripts/chain_stamps.py $O/chain_stamps.bin > $O/stamps.txt 2>&1; head -40 $O/stamps.txt
