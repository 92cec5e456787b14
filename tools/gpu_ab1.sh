set -e
timeout -k 10 300 python -u -m pytest tests/test_gan_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/gan_tests.log 2>&1 || (tail -30 gpurun_out/gan_tests.log; exit 1)
tail -3 gpurun_out/gan_tests.log
timeout -k 10 600 python -u tools/ab_shapes.py tools/variants/base.so tools/variants/cwpe4.so tools/variants/bkw16.so tools/variants/bkw16w3.so > gpurun_out/ab1.log 2>&1
cat gpurun_out/ab1.log
