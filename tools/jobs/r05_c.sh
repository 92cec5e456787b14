#!/bin/bash
# r05c: the r05b job plus the 64-row / dedupe patch variants and the wgrad padding
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
L=./-gan-_amd/libganamd.so
V=tools/variants
export GANAMD_HEARTBEAT=gpurun_out/r05c_heartbeat
AB_SET=patch timeout -k 10 400 python3 -u tools/ab_shapes.py $L $V/p96w4nu.so $V/p96w4.so $V/p96w4mb16nu.so $V/p48w4.so $V/p64.so $V/p16dd.so $L > gpurun_out/r05c_ab.txt 2>&1 &&
AB_SET=patch AB_ACC=1 timeout -k 10 200 python3 -u tools/ab_shapes.py $V/p96w4nu.so $V/p96w4mb16nu.so $V/p48w4.so $V/p64.so $V/p16dd.so > gpurun_out/r05c_acc.txt 2>&1 &&
AB_SET=dg timeout -k 10 300 python3 -u tools/ab_shapes.py $L $V/wide2.so $V/wide1.so $L > gpurun_out/r05c_ab_wide.txt 2>&1 &&
AB_SET=wgrad timeout -k 10 300 python3 -u tools/ab_shapes.py $L $V/wrowpad.so $V/wrowallk.so $L > gpurun_out/r05c_ab_wrow.txt 2>&1 &&
AB_ACC=1 timeout -k 10 200 python3 -u tools/ab_shapes.py $V/wrowallk.so > gpurun_out/r05c_acc_wrow.txt 2>&1 &&
timeout -k 10 1500 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_ops_gpu.py tests/test_critic_gpu.py tests/test_pipeline_gpu.py "tests/test_headline_gpu.py::test_g_step_b16" \
  > gpurun_out/r05c_tests.log 2>&1
