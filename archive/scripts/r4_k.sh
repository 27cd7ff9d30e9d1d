#!/bin/bash
# the two-sweep face passes with one up item per thread (k_face_pp at 576 / 192 threads) vs 512 / 128
# (PAMG_FACE_PP_NT=512): the face tests first, then op = 1 alternating, one box; then the pipelined
# launch's PMC passes (its committed summary predates this round's last kernel-source change)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/r4k; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_face_operator.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { grep -E "FAIL|Error" $O/tests.log | head -20; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do
  echo "== NT 576/192 rep $rep"
  timeout -k 10 200 python scripts/face_probe.py 5 0 2>&1 | grep -v amdgpu.ids || exit 1
  echo "== NT 512/128 rep $rep"
  PAMG_FACE_PP_NT=512 timeout -k 10 200 python scripts/face_probe.py 5 0 2>&1 | grep -v amdgpu.ids || exit 1
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc_pipe_fetch -o run -- python3 $R/scripts/pipe_prof.py 20 > $O/pmc_pipe_fetch.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmc_pipe_write -o run -- python3 $R/scripts/pipe_prof.py 20 > $O/pmc_pipe_write.log 2>&1 || exit 1
echo "all ok"
