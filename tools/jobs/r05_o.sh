#!/bin/bash
# r05o: wide (128x256) vs narrow (128x128) gather tiles on the critic's unscaled GEMMs across batches
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
AB_SET=wide timeout -k 10 600 python3 -u tools/ab_shapes.py ./-gan-_amd/libganamd.so tools/variants/nowide.so ./-gan-_amd/libganamd.so > gpurun_out/r05o_wide.txt 2>&1
