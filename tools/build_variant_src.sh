#!/bin/bash
# Like build_variant.sh, but the unit is compiled from a given source file (an experiment kept out of
# the tree, e.g. under .dev/):   tools/build_variant_src.sh NAME UNIT SRC.hip "-DFLAGS..."
set -e
cd "$(dirname "$0")/.."
mkdir -p tools/variants
P=./-gan-_amd
U=$2
cp "$3" $P/csrc/.ab_src_$U.hip
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -fPIC $4 -I$P/csrc -c $P/csrc/.ab_src_$U.hip -o tools/variants/$1.o
rm -f $P/csrc/.ab_src_$U.hip
OBJS=""
for u in conv_gemm conv_patch conv_wgrad_row conv_small elem gemm_grouped fused data act rng critic; do
  [ "$u" = "$U" ] || OBJS="$OBJS $P/build/$u.hip.o"
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -fPIC -shared -o tools/variants/$1.so tools/variants/$1.o $OBJS
rm tools/variants/$1.o
