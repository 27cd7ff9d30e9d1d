#!/bin/bash
# round 6: op = 1's coarse levels beside level 1 on the handle's second stream -- bitwise against the sequential
# order and the oracle, the fallback with both streams CU-masked, then A/B V-cycles/s (PAMG_FACE_OVERLAP=0 / 1)
set -o pipefail
O=gpurun_out/r6l; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_face_operator.py -x -v --timeout 120 --timeout-method thread \
  -k "beside_level1 or not_coresident or fallback_on_the_per_step or bitwise_the_oracle or agglomerated" \
  -m gpu > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -3 $O/tests.txt
for rep in 1 2 3; do
  for ov in 0 1; do
    PAMG_FACE_OVERLAP=$ov timeout -k 10 120 python -u scripts/face_probe.py 5 0 > $O/ov${ov}_$rep.txt 2>&1 || exit 1
  done
done
grep -H "V-cycles/s\|smooth" $O/ov*_*.txt
