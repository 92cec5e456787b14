#!/bin/bash
# r05g: weight-gradient determinism (NaN-poisoned workspaces), then the row-blocked wgrad parity cases
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -v --timeout 120 --timeout-method thread tests/test_ops_gpu.py \
  -k "wgrad_deterministic or wgrad_row" > gpurun_out/r05g_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|^E " gpurun_out/r05g_tests.log | cut -c1-200
exit $rc
