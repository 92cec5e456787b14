#!/bin/bash
# r05a: LDS-patch conv instance A/B (1 wave/SIMD forms) + accuracy of each variant
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
L=./-gan-_amd/libganamd.so
V=tools/variants
AB_SET=patch timeout -k 10 400 python3 -u tools/ab_shapes.py $L $V/p96w4nu.so $V/p96w4.so $V/p96w4mb16nu.so $V/p48w4.so $L > gpurun_out/r05a_ab.txt 2>&1 || exit 1
AB_SET=patch AB_ACC=1 timeout -k 10 300 python3 -u tools/ab_shapes.py $V/p96w4nu.so $V/p96w4.so $V/p96w4mb16nu.so $V/p48w4.so > gpurun_out/r05a_acc.txt 2>&1
