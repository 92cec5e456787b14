set -e
timeout -k 10 900 python -u tools/ab_shapes.py tools/variants/pf2c.so tools/variants/pf2c.so:GANAMD_WIDE=1 > gpurun_out/ab4.log 2>&1
cat gpurun_out/ab4.log
