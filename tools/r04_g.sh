#!/bin/bash
# Round-4 GPU call: kernel tests, the B=16 mapping-network diagnosis, the headline bench (row-blocked
# wgrad on), model + pipeline tests, per-step kernel breakdowns.
set -o pipefail
mkdir -p gpurun_out
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 300 $T tests/test_ops_gpu.py tests/test_abi.py > gpurun_out/r04g_ops.log 2>&1 &&
timeout -k 10 200 python -u tools/g16_map_diag.py > gpurun_out/r04g_map.log 2>&1 &&
timeout -k 10 400 python -u bench.py --steps 3 --warmup 2 --no-cpu-baseline > gpurun_out/r04g_bench.json 2> gpurun_out/r04g_bench.log &&
timeout -k 10 400 $T tests/test_models_gpu.py tests/test_pipeline_gpu.py > gpurun_out/r04g_models.log 2>&1 &&
timeout -k 10 300 tools/phase_trace.sh r04g > gpurun_out/r04g_phase.log 2>&1
