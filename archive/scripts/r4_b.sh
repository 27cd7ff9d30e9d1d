#!/bin/bash
# Round-4 pass b: the corrected resident call (tests, probe), the face chain as a plain launch (face tests,
# then the face probe under rocprofv3 without the torch import -- the round-3 crash case -- for its exit).
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/${1:-r4b}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_corrected.py tests/test_face_operator.py tests/test_multirank.py tests/test_rccl_self.py -m gpu --maxfail=5 -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?
grep -E "^FAILED|^ERROR" $O/gpu_tests.log | head -20; tail -2 $O/gpu_tests.log
if [ $rc -ne 0 ]; then echo "tests rc $rc"; exit 1; fi
timeout -k 10 300 python scripts/corr_probe.py 5 3 200 > $O/corr_probe.log 2>&1 || { tail -20 $O/corr_probe.log; exit 1; }
cat $O/corr_probe.log
cd /tmp && export TMPDIR=/tmp
PAMG_PROBE_TORCH=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_face -o run -- python3 $R/scripts/face_probe.py 5 0 > $O/prof_face.log 2>&1
echo "face rocprof (chain, plain launch, no torch) exit $?"
grep -v "^[WE]2026" $O/prof_face.log | head -20
