#!/bin/bash
# The face operator's wavefront calls and chain: the face tests (a failed test is reported, a crash
# or hang ends the call), then the event-timed probe, and the probe with the wave / chain phase
# stamps. usage: TAG
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/${1:-wave}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_face_operator.py -m gpu -v --maxfail=3 --timeout 200 --timeout-method thread > $O/face_tests.log 2>&1
rc=$?
grep -E "^FAILED|^ERROR" $O/face_tests.log | head; tail -2 $O/face_tests.log
if [ $rc -ne 0 ]; then echo "tests rc $rc"; exit 1; fi
timeout -k 10 300 python scripts/face_probe.py 5 0 > $O/face_probe.txt 2>&1 || { tail $O/face_probe.txt; exit 1; }
cat $O/face_probe.txt
rm -f $O/wave_stamps.bin $O/chain_stamps.bin
PAMG_WAVE_STAMPS=$O/wave_stamps.bin PAMG_CHAIN_STAMPS=$O/chain_stamps.bin timeout -k 10 300 python scripts/face_probe.py 5 0 > $O/face_probe_stamps.txt 2>&1 || exit 1
python3 scripts/wave_stamps.py $O/wave_stamps.bin > $O/wave_stamps.txt 2>&1; tail -4 $O/wave_stamps.txt
python3 scripts/chain_stamps.py $O/chain_stamps.bin > $O/chain_stamps.txt 2>&1; tail -2 $O/chain_stamps.txt
