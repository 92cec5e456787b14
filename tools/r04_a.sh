#!/bin/bash
# Round-4 first GPU call: B=16 G-step gradient diagnosis (default build and plain-fp32-MFMA variant),
# the critic engine tests incl. threads + capture, and peak HBM vs the warm-up count.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/g16_grad_diag.py gpu > gpurun_out/r04a_g16.log 2>&1 &&
G16_TAG=nosplit GANAMD_SO=$(realpath tools/variants/nosplit.so) timeout -k 10 300 python -u tools/g16_grad_diag.py gpu >> gpurun_out/r04a_g16.log 2>&1 &&
timeout -k 10 600 python -u -m pytest tests/test_critic_gpu.py -x -v -k "engine" --timeout 300 --timeout-method thread > gpurun_out/r04a_critic.log 2>&1 &&
timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras > gpurun_out/r04a_bench_w1.json 2> gpurun_out/r04a_bench_w1.log &&
timeout -k 10 400 python -u bench.py --steps 3 --warmup 4 --no-cpu-baseline --no-extras > gpurun_out/r04a_bench_w4.json 2> gpurun_out/r04a_bench_w4.log
