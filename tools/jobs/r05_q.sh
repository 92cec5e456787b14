#!/bin/bash
# r05q: configs 4 (lazy GP + R1/R2, bf16, B=128) and 5 (progan pair) at the round-5 build
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python3 bench.py --config lazy --no-cpu-baseline > gpurun_out/r05q_lazy.log 2>&1 &&
timeout -k 10 400 python3 bench.py --config progan --no-cpu-baseline > gpurun_out/r05q_progan.log 2>&1
rc=$?
for f in gpurun_out/r05q_lazy.log gpurun_out/r05q_progan.log; do grep '^{"metric' $f | cut -c1-220; done
exit $rc
