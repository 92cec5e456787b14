#!/bin/bash
# Round-4 GPU call C: patch-off A/B bench, peak HBM vs the warm-up count, config-4 bf16 tests.
set -o pipefail
mkdir -p gpurun_out
T="python -u -m pytest -x -v --timeout 900 --timeout-method thread"
timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras --patch off > gpurun_out/r04c_bench_off.json 2> gpurun_out/r04c_bench_off.log &&
timeout -k 10 400 python -u bench.py --steps 3 --warmup 4 --no-cpu-baseline --no-extras > gpurun_out/r04c_bench_w4.json 2> gpurun_out/r04c_bench_w4.log &&
timeout -k 10 900 $T tests/test_headline_gpu.py tests/test_critic_gpu.py -k "bf16" > gpurun_out/r04c_bf16.log 2>&1
