set -e
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu 2>&1 | tail -3
echo NEW; timeout -k 10 120 python -u tools/resample_micro.py 2>&1 | grep -v amdgpu.ids
# A/B: build the previous library into tmp_ab/libold.so and add: GANAMD_SO=$PWD/tmp_ab/libold.so python tools/resample_micro.py
timeout -k 10 300 python -u bench.py --steps 3 --warmup 2 --no-cpu-baseline 2>/dev/null
