#!/bin/bash
# r05r: the full GEMM census of one iteration (every distinct conv GEMM timed alone)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
GANAMD_CENSUS_OUT=gpurun_out/r05_census_full.txt timeout -k 10 500 python3 bench.py --no-cpu-baseline > gpurun_out/r05r_bench.log 2>&1
