#!/bin/bash
# r05fin: the by-value all-kernel-rows wgrad in tree -- determinism + parity gates, generator /
# pipeline / DP tests, then the headline bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ops_gpu.py \
  tests/test_pipeline_gpu.py tests/test_headline_gpu.py tests/test_dp_gpu.py tests/test_critic_gpu.py > gpurun_out/r05fin_tests.log 2>&1 || { tail -n 8 gpurun_out/r05fin_tests.log; exit 1; }
tail -n 1 gpurun_out/r05fin_tests.log
timeout -k 10 300 python3 bench.py --no-cpu-baseline > gpurun_out/r05fin_bench.log 2>&1 && grep '^{"metric' gpurun_out/r05fin_bench.log | cut -c1-230
