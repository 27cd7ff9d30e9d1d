#!/bin/bash
# Build A/B variants of libpamg into scripts/ablibs (run here, on the CPU; the GPU box only
# loads them through PAMG_LIB, scripts/ab2.sh). Usage: build_ab.sh NAME [hipcc -D flags] ...
#   e.g. build_ab.sh a_base  &&  build_ab.sh b_tail2 -DPAMG_TAIL_PRIO=2
set -eo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
name=$1
shift
tmp=$(mktemp -d /tmp/pamg_ab_XXXX)
cp -r "$ROOT/p-a_multigrids_amd" "$ROOT/include" "$tmp/"
cd "$tmp/p-a_multigrids_amd"
rm -rf build pamg/libpamg.so
make -j8 pamg/libpamg.so HIPCC="/opt/rocm/bin/hipcc $*" > "$tmp/build.log" 2>&1
mkdir -p "$ROOT/scripts/ablibs"
cp pamg/libpamg.so "$ROOT/scripts/ablibs/$name.so"
rm -rf "$tmp"
echo "built scripts/ablibs/$name.so ($*)"
