#!/bin/bash
# Round-4 GPU call: patch conv with the block's scales staged in LDS and the weight / patch loads
# issued after each tap's products (A/B vs tools/variants/base.so = HEAD before the change), the
# patch / conv kernel tests, and the headline bench per library.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/r04p_ab.log
for A in "--op fwd --B 256 --cin 96 --H 64 --cout 96 --k 5 --pad 2 --scaled --reps 10" \
         "--op fwd --B 64 --cin 96 --H 64 --cout 96 --k 5 --pad 2 --scaled --reps 10" \
         "--op fwd --B 256 --cin 48 --H 64 --cout 48 --k 5 --pad 2 --scaled --reps 10" \
         "--op fwd --B 256 --cin 48 --H 64 --cout 48 --k 3 --pad 1 --scaled --reps 10" \
         "--op fwd --B 256 --cin 96 --H 32 --cout 96 --k 5 --pad 2 --scaled --reps 10" \
         "--op dgrad --B 64 --cin 96 --H 64 --cout 96 --k 5 --pad 2 --scaled --reps 10" \
         "--op fwd --B 128 --cin 64 --H 64 --cout 64 --k 3 --pad 1 --reps 10"; do
  for SO in tools/variants/base.so -gan-_amd/libganamd.so; do
    echo "== $SO $A" >> gpurun_out/r04p_ab.log
    GANAMD_SO=$(realpath -- $SO) timeout -k 10 120 python3 tools/gemm_micro.py $A >> gpurun_out/r04p_ab.log 2>&1 || exit 1
  done
done
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 300 $T tests/test_ops_gpu.py -k "patch or split6 or modconv or conv_fwd" > gpurun_out/r04p_ops.log 2>&1 &&
STEPS=3 timeout -k 10 700 bash tools/ab_lib.sh r04p tools/variants/base.so -gan-_amd/libganamd.so tools/variants/base.so -gan-_amd/libganamd.so > /dev/null 2>&1 &&
timeout -k 10 300 tools/pmc_traffic.sh > gpurun_out/r04p_pmc.log 2>&1 &&
rm -rf /tmp/gpt && timeout -k 10 400 rocprofv3 --kernel-trace -d /tmp/gpt -o run --output-format csv -- python3 tools/graph_phase_trace.py > gpurun_out/r04p_gpt.log 2>&1 &&
python3 tools/graph_phase_trace.py --analyse $(find /tmp/gpt -name "*kernel_trace.csv") > gpurun_out/r04p_phases.txt &&
GANAMD_CENSUS_OUT=gpurun_out/r04p_census.txt timeout -k 10 400 python -u bench.py --steps 3 --warmup 2 --no-cpu-baseline > gpurun_out/r04p_bench.json 2> gpurun_out/r04p_bench.log
