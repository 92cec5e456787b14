#!/bin/bash
# progan DP diagnosis: 2 ranks with the fake-batch overlap, 4 ranks without it.
mkdir -p gpurun_out
T="python -u -m pytest -x -v --timeout 600 --timeout-method thread"
GANAMD_TEST_PROGAN_WORLD=2 timeout -k 10 400 $T tests/test_dp_gpu.py -k progan > gpurun_out/r04y_w2.log 2>&1
GANAMD_TEST_PROGAN_OVERLAP=0 timeout -k 10 400 $T tests/test_dp_gpu.py -k progan > gpurun_out/r04y_noov.log 2>&1
exit 0
