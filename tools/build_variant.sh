#!/bin/bash
# Build an A/B variant of the product library with extra compile flags:
#   tools/build_variant.sh NAME [-DFLAG ...]  ->  metagenomics_amd/lib/variants/NAME.so
# (tools/ab_libs.sh runs every variant against the default build on one box)
# SRC=<file> compiles another mg_kernels.hip (e.g. `git show HEAD:...` of the
# last commit) in place of the working tree's.
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; shift
B=$ROOT/metagenomics_amd/build/variants/$NAME
mkdir -p $B $ROOT/metagenomics_amd/lib/variants
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I$ROOT/include -Wno-unused-result "$@" \
  -I$ROOT/metagenomics_amd/csrc/device -c ${SRC:-$ROOT/metagenomics_amd/csrc/device/mg_kernels.hip} -o $B/mg_kernels.o
O=$ROOT/metagenomics_amd/build
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -pthread -o $ROOT/metagenomics_amd/lib/variants/$NAME.so \
  $B/mg_kernels.o $O/mg_dataset.o $O/mg_host.o $O/mg_graph.o $O/mg_unitig.o $O/mg_parse.o $O/mg_rdzv.o
