#!/bin/bash
# round 5: the sync poll spins first (default 5 ms) -- the exchange probe at an N = 8 rank's shape again
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/r5d; mkdir -p $O
timeout -k 10 200 python scripts/xe_probe.py > $O/xe_early.txt 2>&1 || { tail $O/xe_early.txt; exit 1; }
PAMG_EARLY_XC=0 timeout -k 10 200 python scripts/xe_probe.py > $O/xe_after.txt 2>&1 || { tail $O/xe_after.txt; exit 1; }
PAMG_SYNC_SPIN_MS=0 timeout -k 10 200 python scripts/xe_probe.py > $O/xe_early_sleep.txt 2>&1 || { tail $O/xe_early_sleep.txt; exit 1; }
for f in xe_early xe_after xe_early_sleep; do echo "== $f"; grep -v -E "amdgpu.ids|version|Hostname|Librccl" $O/$f.txt; done
echo "all ok"
