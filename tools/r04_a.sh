#!/bin/bash
# Round-4 first GPU call: B=16 G-step gradient diagnosis (default build and plain-fp32-MFMA variant),
# the critic engine tests incl. threads + capture, the new parity tests, peak HBM vs the warm-up count.
set -o pipefail
mkdir -p gpurun_out
T="python -u -m pytest -x -v --timeout 900 --timeout-method thread"
timeout -k 10 300 python -u tools/g16_grad_diag.py gpu > gpurun_out/r04a_g16.log 2>&1 &&
G16_TAG=nosplit G16_PATCH=0 GANAMD_SO=$(realpath tools/variants/nosplit.so) timeout -k 10 300 python -u tools/g16_grad_diag.py gpu >> gpurun_out/r04a_g16.log 2>&1 &&
timeout -k 10 900 $T tests/test_critic_gpu.py tests/test_dp_gpu.py tests/test_ops_gpu.py -k "engine or progan or split6" > gpurun_out/r04a_tests.log 2>&1 &&
timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras > gpurun_out/r04a_bench_w1.json 2> gpurun_out/r04a_bench_w1.log &&
timeout -k 10 400 python -u bench.py --steps 3 --warmup 4 --no-cpu-baseline --no-extras > gpurun_out/r04a_bench_w4.json 2> gpurun_out/r04a_bench_w4.log &&
timeout -k 10 900 $T tests/test_headline_gpu.py tests/test_critic_gpu.py -k "bf16" > gpurun_out/r04a_bf16.log 2>&1
