#!/bin/bash
# round 5 (session 2): timing diagnostic -- the per-wave chain's phases with and without its word stores
# (PAMG_DIAG_CHAIN_NOWORDS=1: results wrong, stamps only)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/r5al; mkdir -p $O
for p in 0 1; do
  rm -f $O/st$p.bin
  PAMG_DIAG_CHAIN_NOWORDS=$p PAMG_CHAIN_STAMPS=$O/st$p.bin timeout -k 10 200 python scripts/face_probe.py 5 0 > $O/probe_st$p.txt 2>&1 || { tail $O/probe_st$p.txt; exit 1; }
  python scripts/chain_stamps.py $O/st$p.bin > $O/st$p.txt
  echo "stamps nowords=$p"; grep 'run  59' $O/st$p.txt | tail -3
done
echo "all ok"
