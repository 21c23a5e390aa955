#!/bin/bash
# CPU test suite against the ASan + UBSan build of the host C++ (make -C
# metagenomics_amd/csrc asan).  Leak checking is off: the Python interpreter and
# torch are not instrumented and hold allocations until exit.
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
make -s -C "$ROOT/metagenomics_amd/csrc" asan
RT=$(/opt/rocm/lib/llvm/bin/clang++ -print-file-name=libclang_rt.asan-x86_64.so)
export MG_LIB="$ROOT/metagenomics_amd/lib/asan/libmgovl.so"
export ASAN_OPTIONS=detect_leaks=0:halt_on_error=1:abort_on_error=1
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
LD_PRELOAD="$RT" python -m pytest "$ROOT/tests" -x -q -m "not gpu" -p no:cacheprovider "$@"
