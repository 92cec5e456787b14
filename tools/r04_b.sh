#!/bin/bash
# Round-4 GPU call B: the split6 LDS-patch conv and row-blocked wgrad (correctness first), the
# headline bench with them (full extras), the B=16 G-step gradient diagnosis, the engine / DP tests.
set -o pipefail
mkdir -p gpurun_out
T="python -u -m pytest -x -v --timeout 900 --timeout-method thread"
timeout -k 10 600 $T tests/test_ops_gpu.py -k "patch or split6 or wgrad or conv_fwd_dgrad" > gpurun_out/r04b_kernel_tests.log 2>&1 &&
timeout -k 10 500 python -u bench.py --steps 3 --warmup 2 --no-cpu-baseline > gpurun_out/r04b_bench.json 2> gpurun_out/r04b_bench.log &&
timeout -k 10 300 python -u tools/g16_grad_diag.py gpu > gpurun_out/r04b_g16.log 2>&1 &&
G16_TAG=nosplit G16_PATCH=0 GANAMD_SO=$(realpath tools/variants/nosplit.so) timeout -k 10 300 python -u tools/g16_grad_diag.py gpu >> gpurun_out/r04b_g16.log 2>&1 &&
timeout -k 10 900 $T tests/test_critic_gpu.py tests/test_dp_gpu.py -k "engine or progan" > gpurun_out/r04b_tests.log 2>&1
