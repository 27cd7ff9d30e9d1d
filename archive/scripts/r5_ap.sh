#!/bin/bash
# round 5 (session 3): the chain launches gated on the stream (the host reads their reports back at the call's end
# instead of waiting for each) and the coarsest residual only in a call's last cycle: face tests (the CU-masked
# fallback with the gate and without), probe A/B against the previous build (scripts/ablibs/base.so)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/r5ap; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_face_operator.py -k not_coresident > $O/t_fb.log 2>&1 || { tail -30 $O/t_fb.log; exit 1; }
grep -E "PASS|FAIL" $O/t_fb.log
PAMG_CHAIN_GATE=0 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_face_operator.py -k not_coresident > $O/t_fb0.log 2>&1 || { tail -30 $O/t_fb0.log; exit 1; }
tail -1 $O/t_fb0.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_face_operator.py > $O/t_face.log 2>&1 || { tail -30 $O/t_face.log; exit 1; }
tail -1 $O/t_face.log
run() {   # tag lib gate
  if [ $2 = base ]; then L=$R/scripts/ablibs/base.so; else L=; fi
  PAMG_LIB=$L PAMG_CHAIN_GATE=$3 timeout -k 10 200 python scripts/face_probe.py 5 0,1 > $O/probe_$1.txt 2>&1 || { tail $O/probe_$1.txt; exit 1; }
  echo "$1"; grep -E "V-cycles" $O/probe_$1.txt
}
for i in 1 2; do
  run base_$i base 1 || exit 1
  run nogate_$i new 0 || exit 1
  run gate_$i new 1 || exit 1
done
echo "all ok"
