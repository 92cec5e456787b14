#!/bin/bash
# Build an A/B variant of libganamd.so with extra compile flags on conv_gemm.hip (the other objects
# come from the in-tree build):   tools/build_variant.sh NAME "-DFLAG=1 ..."  ->  tools/variants/NAME.so
set -e
cd "$(dirname "$0")/.."
mkdir -p tools/variants
P=./-gan-_amd
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -fPIC $2 -c $P/csrc/conv_gemm.hip -o tools/variants/$1.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -fPIC -shared -o tools/variants/$1.so tools/variants/$1.o \
  $P/build/elem.hip.o $P/build/gemm_grouped.hip.o $P/build/fused.hip.o $P/build/data.hip.o $P/build/act.hip.o
rm tools/variants/$1.o
