#!/bin/bash
# Build an A/B variant of libganamd.so with extra compile flags on one translation unit (the other
# objects come from the in-tree build):
#   UNIT=conv_patch tools/build_variant.sh NAME "-DFLAG=1 ..." [GIT_REV]
#   -> tools/variants/NAME.so   (UNIT defaults to conv_gemm; GIT_REV: compile the unit as of that revision)
set -e
cd "$(dirname "$0")/.."
mkdir -p tools/variants
P=./-gan-_amd
U=${UNIT:-conv_gemm}
SRC=$P/csrc/$U.hip
if [ -n "$3" ]; then
  SRC=$P/csrc/.ab_rev_$U.hip
  git show "$3:-gan-_amd/csrc/$U.hip" > "$SRC"
fi
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -fPIC $2 -c $SRC -o tools/variants/$1.o
[ -n "$3" ] && rm -f "$SRC"
OBJS=""
for u in conv_gemm conv_patch conv_wgrad_row conv_small elem gemm_grouped fused data act rng critic; do
  [ "$u" = "$U" ] || OBJS="$OBJS $P/build/$u.hip.o"
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -fPIC -shared -o tools/variants/$1.so tools/variants/$1.o $OBJS
rm tools/variants/$1.o
