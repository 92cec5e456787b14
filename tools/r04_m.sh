#!/bin/bash
# Round-4 GPU call: 12-wave 96-row patch conv (A/B vs the 8-wave build tools/variants/unroll.so),
# kernel tests, the penalty sweeps on a second stream (model / pipeline / critic tests), bench.
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/r04m_ab.log
for A in "--op fwd --B 256 --cin 96 --H 64 --cout 96 --k 5 --pad 2 --scaled --reps 10" \
         "--op fwd --B 64 --cin 96 --H 64 --cout 96 --k 3 --pad 1 --scaled --reps 10" \
         "--op dgrad --B 64 --cin 96 --H 64 --cout 96 --k 5 --pad 2 --scaled --reps 10" \
         "--op fwd --B 128 --cin 64 --H 64 --cout 64 --k 3 --pad 1 --reps 10"; do
  for SO in tools/variants/unroll.so -gan-_amd/libganamd.so; do
    echo "== $SO $A" >> gpurun_out/r04m_ab.log
    GANAMD_SO=$(realpath -- $SO) timeout -k 10 120 python3 tools/gemm_micro.py $A >> gpurun_out/r04m_ab.log 2>&1 || exit 1
  done
done
T="python -u -m pytest -x -v --timeout 600 --timeout-method thread"
timeout -k 10 300 $T tests/test_ops_gpu.py -k "patch or split6 or modconv or conv_fwd" > gpurun_out/r04m_ops.log 2>&1 &&
timeout -k 10 500 $T tests/test_pipeline_gpu.py tests/test_models_gpu.py tests/test_critic_gpu.py > gpurun_out/r04m_tests.log 2>&1 &&
timeout -k 10 400 python -u bench.py --steps 3 --warmup 2 --no-cpu-baseline > gpurun_out/r04m_bench.json 2> gpurun_out/r04m_bench.log
