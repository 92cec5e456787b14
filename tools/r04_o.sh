#!/bin/bash
# Round-4 GPU call: XCD-aware patch conv order + fp32-body removal (conv / split6 / patch kernel
# tests, PMC traffic of the probe launch), the per-phase attributed breakdown of the captured
# graphs (tools/graph_phase_trace.py), and the bench with the full GEMM census.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 400 $T tests/test_ops_gpu.py tests/test_abi.py > gpurun_out/r04o_ops.log 2>&1 &&
timeout -k 10 300 tools/pmc_traffic.sh > gpurun_out/r04o_pmc.log 2>&1 &&
rm -rf /tmp/gpt && timeout -k 10 400 rocprofv3 --kernel-trace -d /tmp/gpt -o run --output-format csv -- python3 tools/graph_phase_trace.py > gpurun_out/r04o_gpt.log 2>&1 &&
python3 tools/graph_phase_trace.py --analyse $(find /tmp/gpt -name "*kernel_trace.csv") > gpurun_out/r04o_phases.txt &&
GANAMD_CENSUS_OUT=gpurun_out/r04o_census.txt timeout -k 10 400 python -u bench.py --steps 3 --warmup 2 --no-cpu-baseline > gpurun_out/r04o_bench.json 2> gpurun_out/r04o_bench.log
