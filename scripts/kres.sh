#!/bin/bash
# Kernel resource summary of pamg_vcycle.hip (VGPRs, scratch, occupancy, LDS) for kernels matching $1.
# usage: scripts/kres.sh REGEX [extra hipcc -D flags]
cd "$(dirname "$0")/../p-a_multigrids_amd"
pat=$1; shift
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -I../include -DPAMG_STAMPS=0 -DPAMG_NT=3 "$@" \
  -Rpass-analysis=kernel-resource-usage -c csrc/${KRES_SRC:-pamg_vcycle.hip} -o /tmp/kres_$$.o 2>&1 | python3 -c '
import re, sys
pat = re.compile(sys.argv[1]); cur = None; rows = {}
for line in sys.stdin:
    m = re.search(r"Function Name: (\S+)", line)
    if m: cur = m.group(1); rows[cur] = {}; continue
    m = re.search(r"remark:\s+(VGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]): (\d+)", line)
    if m and cur: rows[cur][m.group(1).split()[0]] = m.group(2)
for k, v in rows.items():
    if pat.search(k): print(k[22:90].ljust(70), "vgpr", v.get("VGPRs"), "scratch", v.get("ScratchSize"), "occ", v.get("Occupancy"), "lds", v.get("LDS"))
' "$pat"
rm -f /tmp/kres_$$.o
