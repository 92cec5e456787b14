#!/bin/bash
# Round-4 GPU call: the practical split6 ceiling (bare bf16 MFMA loops on random vs zero operands at
# 1..4 waves/SIMD, in-kernel clock), then the round's committed evidence (tools/round_profile.sh r04).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 tools/variants/mfma_peak_bf16 > gpurun_out/r04r_mfma_bf16.txt 2>&1 &&
timeout -k 10 1000 bash tools/round_profile.sh r04 > gpurun_out/r04r_profile.log 2>&1
