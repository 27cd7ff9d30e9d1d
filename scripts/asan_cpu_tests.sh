#!/bin/bash
# Host sanitizer pass (AddressSanitizer + UndefinedBehaviorSanitizer) over the CPU test suite: the
# library's host code (mesh reader, setup tables, halo plan, VTU writer, C-ABI; make -C
# p-a_multigrids_amd asan) and the oracle (make -C oracle asan) instrumented, loaded by the tests through
# PAMG_LIB / ORACLE_LIB with the clang ASan runtime preloaded into the (uninstrumented) interpreter.
# Runs here, on the CPU (the GPU box refuses GPU sanitizer runs; nothing here touches a GPU).
set -eo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
make -s -C "$ROOT/p-a_multigrids_amd" -j8 asan
make -s -C "$ROOT/oracle" asan
RT=$(/opt/rocm/lib/llvm/bin/clang -print-file-name=libclang_rt.asan-x86_64.so)
cd "$ROOT"
# leaks: the interpreter itself is not instrumented and keeps its allocations until exit
LD_PRELOAD=$RT ASAN_OPTIONS=detect_leaks=0:abort_on_error=1:halt_on_error=1 \
UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 \
PAMG_LIB="$ROOT/p-a_multigrids_amd/build_asan/libpamg.so" ORACLE_LIB="$ROOT/oracle/_build/liborc_asan.so" \
    python -m pytest tests -q -m "not gpu" -p no:cacheprovider "$@"
