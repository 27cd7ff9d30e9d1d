#!/bin/bash
# round 5 (session 2): the per-wave chain's halo words as 16-byte sc1 stores of whole t_overlap rows (the wave's rows
# cut into chunks, read back from the tile in LDS) instead of three 8-byte stores per face and item-1 lane: face
# tests, the chain's stamps, probe A/B against the previous build (scripts/ablibs/base.so)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/r5am; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_face_operator.py > $O/t_face.log 2>&1 || { tail -30 $O/t_face.log; exit 1; }
tail -1 $O/t_face.log
for b in base new; do
  if [ $b = base ]; then L=$R/scripts/ablibs/base.so; else L=; fi
  rm -f $O/st_$b.bin
  PAMG_LIB=$L PAMG_CHAIN_STAMPS=$O/st_$b.bin timeout -k 10 200 python scripts/face_probe.py 5 0 > $O/probe_st_$b.txt 2>&1 || { tail $O/probe_st_$b.txt; exit 1; }
  python scripts/chain_stamps.py $O/st_$b.bin > $O/st_$b.txt
  echo "stamps $b"; grep 'run  59' $O/st_$b.txt | tail -2
done
for i in 1 2; do
  for b in base new; do
    if [ $b = base ]; then L=$R/scripts/ablibs/base.so; else L=; fi
    PAMG_LIB=$L timeout -k 10 200 python scripts/face_probe.py 5 0,1 > $O/probe_${b}_$i.txt 2>&1 || { tail $O/probe_${b}_$i.txt; exit 1; }
    echo "$b rep $i"; grep -E "V-cycles|smooth " $O/probe_${b}_$i.txt
  done
done
echo "all ok"
