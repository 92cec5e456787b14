#!/bin/bash
# Round-4 GPU call: the B=16 mapping-network diagnosis with the isolated BN backward check.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/g16_map_diag.py > gpurun_out/r04i_map.log 2>&1
