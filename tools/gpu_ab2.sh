set -e
timeout -k 10 900 python -u tools/ab_shapes.py tools/variants/base.so tools/variants/base.so:GANAMD_CONV_LDS_PAD=28672 tools/variants/base.so:GANAMD_WGRAD_LDS_PAD=28672 tools/variants/base.so:GANAMD_CONV_LDS_PAD=60000,GANAMD_WGRAD_LDS_PAD=60000 > gpurun_out/ab2.log 2>&1
cat gpurun_out/ab2.log
