#!/bin/bash
# Build an A/B variant of libganamd.so with extra compile flags on conv_gemm.hip (the other objects
# come from the in-tree build):   tools/build_variant.sh NAME "-DFLAG=1 ..." [GIT_REV]
#   -> tools/variants/NAME.so   (GIT_REV: compile conv_gemm.hip as of that revision instead)
set -e
cd "$(dirname "$0")/.."
mkdir -p tools/variants
P=./-gan-_amd
SRC=$P/csrc/conv_gemm.hip
if [ -n "$3" ]; then
  SRC=$P/csrc/.ab_rev_conv_gemm.hip
  git show "$3:-gan-_amd/csrc/conv_gemm.hip" > "$SRC"
fi
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -fPIC $2 -c $SRC -o tools/variants/$1.o
[ -n "$3" ] && rm -f "$SRC"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -fPIC -shared -o tools/variants/$1.so tools/variants/$1.o \
  $P/build/conv_patch.hip.o $P/build/conv_wgrad_row.hip.o $P/build/elem.hip.o $P/build/gemm_grouped.hip.o $P/build/fused.hip.o $P/build/data.hip.o $P/build/act.hip.o \
  $P/build/rng.hip.o $P/build/critic.hip.o
rm tools/variants/$1.o
