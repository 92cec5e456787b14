#!/bin/bash
# r05t: forward / input-gradient / weight-gradient determinism across the conv kernels
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest -v --timeout 120 --timeout-method thread tests/test_ops_gpu.py \
  -k "deterministic" > gpurun_out/r05t_tests.log 2>&1
rc=$?
grep -E "FAILED|passed|failed|^E " gpurun_out/r05t_tests.log | cut -c1-200 | head -20
exit $rc
