set -e
timeout -k 10 900 python -u tools/ab_shapes.py tools/variants/base.so tools/variants/pf2b.so tools/variants/pf2b.so:GANAMD_CONV_LDS_PAD=28672 > gpurun_out/ab3.log 2>&1
cat gpurun_out/ab3.log
