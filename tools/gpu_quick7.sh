set -e
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/tests.log 2>&1 || (grep -E "FAIL|Error|assert" gpurun_out/tests.log | head; tail -30 gpurun_out/tests.log; exit 1)
tail -1 gpurun_out/tests.log
for v in 1 0 1; do GANAMD_WGRAD_TP=$v timeout -k 10 600 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-extras > gpurun_out/b.log 2>&1; python3 -c "import json; d=json.loads(open('gpurun_out/b.log').read().strip().splitlines()[-1]); print('tp=$v', round(d['value'],2), round(d['ms_per_step'],1))"; done
