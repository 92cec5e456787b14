#!/bin/bash
# Round-4 GPU call: the headline bench (full extras), the B=16 G-step diagnosis, one-iteration profile.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --steps 3 --warmup 2 --no-cpu-baseline > gpurun_out/r04e_bench.json 2> gpurun_out/r04e_bench.log &&
timeout -k 10 300 python -u tools/g16_grad_diag.py gpu > gpurun_out/r04e_g16.log 2>&1 &&
timeout -k 10 400 tools/prof_iter.sh r04e > gpurun_out/r04e_prof.log 2>&1
