#!/bin/bash
# round 5 (session 2): the per-wave chain's phases (PAMG_CHAIN_STAMPS) with the flags polled 64 at a time (0) or all at
# once (PAMG_CHAIN_POLL=1); face tests with POLL=1; probe A/B without stamps
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/r5x; mkdir -p $O
PAMG_CHAIN_POLL=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_face_operator.py > $O/t_face.log 2>&1 || { tail -30 $O/t_face.log; exit 1; }
tail -1 $O/t_face.log
for p in 0 1; do
  rm -f $O/st$p.bin
  PAMG_CHAIN_POLL=$p PAMG_CHAIN_STAMPS=$O/st$p.bin timeout -k 10 200 python scripts/face_probe.py 5 0 > $O/probe_st$p.txt 2>&1 || { tail $O/probe_st$p.txt; exit 1; }
  python scripts/chain_stamps.py $O/st$p.bin > $O/st$p.txt
  echo "stamps poll=$p"; grep 'run  59' $O/st$p.txt | tail -3
done
for i in 1 2; do
  for p in 0 1; do
    PAMG_CHAIN_POLL=$p timeout -k 10 200 python scripts/face_probe.py 5 0,1 > $O/probe_p${p}_$i.txt 2>&1 || { tail $O/probe_p${p}_$i.txt; exit 1; }
    echo "poll=$p rep $i"; grep -E "V-cycles|smooth " $O/probe_p${p}_$i.txt
  done
done
echo "all ok"
