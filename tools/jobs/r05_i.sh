#!/bin/bash
# r05i: where the row-blocked wgrad goes wrong (96 -> 96 3x3 64x64 B=8 scaled), this build and the round-4 kernel
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 python3 -u tools/wgrad_race.py 8 96 96 64 3 1 20 > gpurun_out/r05i_base.log 2>&1 &&
GANAMD_SO=tools/variants/wrow_r04.so timeout -k 10 120 python3 -u tools/wgrad_race.py 8 96 96 64 3 1 20 > gpurun_out/r05i_r04.log 2>&1 &&
timeout -k 10 120 python3 -u tools/wgrad_race.py 8 96 96 64 3 0 20 > gpurun_out/r05i_base_unscaled.log 2>&1 &&
timeout -k 10 120 python3 -u tools/wgrad_race.py 8 128 128 32 3 0 20 > gpurun_out/r05i_base_128.log 2>&1
