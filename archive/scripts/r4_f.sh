#!/bin/bash
# Round-4 pass f: the face operator's fused calls on partitions (an exchange per sweep into the snapshot
# buffer it reads): face tests, then the per-rank partition timing.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/${1:-r4f}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_face_operator.py tests/test_corrected.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?
grep -E "^FAILED|^ERROR" $O/gpu_tests.log | head; tail -2 $O/gpu_tests.log
if [ $rc -ne 0 ]; then grep -B5 -A40 "Error\|assert" $O/gpu_tests.log | head -80; exit 1; fi
timeout -k 10 300 python scripts/face_strong_probe.py 5 10 > $O/face_strong.log 2>&1 || { tail -5 $O/face_strong.log; exit 1; }
grep -v amdgpu.ids $O/face_strong.log
