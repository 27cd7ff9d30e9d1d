#!/bin/bash
# round 5 (session 2): the chain's polled workgroups from LDS (no dependent nb_list load in front of a sweep's first
# poll): face tests,
# stamps and probe A/B against the previous build (scripts/ablibs/base.so)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/r5ao; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_face_operator.py > $O/t_face.log 2>&1 || { tail -30 $O/t_face.log; exit 1; }
tail -1 $O/t_face.log
run() {   # tag lib pipe
  if [ $2 = base ]; then L=$R/scripts/ablibs/base.so; else L=; fi
  PAMG_LIB=$L PAMG_CHAIN_POLL_PIPE=$3 timeout -k 10 200 python scripts/face_probe.py 5 0,1 > $O/probe_$1.txt 2>&1 || { tail $O/probe_$1.txt; exit 1; }
  echo "$1"; grep -E "V-cycles|smooth " $O/probe_$1.txt
}
for v in "base base 0" "lds new 0"; do
  set -- $v
  rm -f $O/st_$1.bin
  if [ $2 = base ]; then L=$R/scripts/ablibs/base.so; else L=; fi
  PAMG_LIB=$L PAMG_CHAIN_POLL_PIPE=$3 PAMG_CHAIN_STAMPS=$O/st_$1.bin timeout -k 10 200 python scripts/face_probe.py 5 0 > $O/probe_st_$1.txt 2>&1 || exit 1
  python scripts/chain_stamps.py $O/st_$1.bin > $O/st_$1.txt
  echo "stamps $1"; grep 'run  59' $O/st_$1.txt | tail -2
done
for i in 1 2; do
  run base_$i base 0 || exit 1
  run lds_$i new 0 || exit 1

done
echo "all ok"
