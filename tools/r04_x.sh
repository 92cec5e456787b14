#!/bin/bash
# Round-4 GPU call: progan DP diagnosis -- uninitialised-workspace probe (NaN-poisoned allocator), and the
# 4-rank test with the LDS-patch conv / row-blocked wgrad off (mask 0) and on (default).
set -o pipefail
mkdir -p gpurun_out
T="python -u -m pytest -x -v --timeout 600 --timeout-method thread"
timeout -k 10 300 python3 -u tools/progan_dp_diag.py 1 poison > gpurun_out/r04x_diag.log 2>&1 &&
GANAMD_TEST_PATCH_MASK=0 timeout -k 10 400 $T tests/test_dp_gpu.py -k progan > gpurun_out/r04x_dp_mask0.log 2>&1
GANAMD_TEST_PATCH_MASK=3 timeout -k 10 400 $T tests/test_dp_gpu.py -k progan > gpurun_out/r04x_dp_mask3.log 2>&1
exit 0
