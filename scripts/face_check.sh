#!/bin/bash
# Face-operator GPU pass: its tests (a failed test is reported, a crash or hang ends the call), then
# the event-timed probe. usage: face_check.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-face}
O=$R/gpurun_out/$TAG
mkdir -p $O && cd $R
timeout -k 10 600 python -u -m pytest tests/test_face_operator.py tests/test_rccl_self.py -m gpu -v --maxfail=5 --timeout 200 --timeout-method thread > $O/face_tests.log 2>&1
rc=$?
grep -E "^FAILED|^ERROR" $O/face_tests.log | head; tail -2 $O/face_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests rc $rc"; exit 1; fi
timeout -k 10 300 python scripts/face_probe.py 5 0 > $O/face_probe.txt 2>&1 || { tail $O/face_probe.txt; exit 1; }
cat $O/face_probe.txt
rm -f $O/chain_stamps.bin
PAMG_CHAIN_STAMPS=$O/chain_stamps.bin timeout -k 10 300 python scripts/face_probe.py 5 0 > $O/face_probe_stamps.txt 2>&1 || exit 1
python3 scripts/chain_stamps.py $O/chain_stamps.bin | sort | uniq -c | sort -rn | head -8
