set -e
for b in 256 512 768 1024; do timeout -k 10 120 tools/variants/mfma_peak_rand $b; done > gpurun_out/mfma_ceiling2.txt 2>&1
cat gpurun_out/mfma_ceiling2.txt
