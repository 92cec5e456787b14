#!/bin/bash
# r05m: memory of the 2-rank B=64 DP graph test after the critic / data modules (full-suite order)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
DP_MEMLOG=1 timeout -k 10 600 python3 -u -m pytest -v -s -x --timeout 300 --timeout-method thread tests/test_critic_gpu.py tests/test_data.py \
  "tests/test_dp_gpu.py::test_dp_graph_iteration_matches_shard_mean" > gpurun_out/r05m.log 2>&1
rc=$?
grep -E "referrer|largest live|\[mem\]|before the ranks|rank 0: peak|graph-mode DP|passed|failed|OutOfMemory" gpurun_out/r05m.log | cut -c1-300
exit $rc
