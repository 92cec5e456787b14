set -e
for o in "" "--no-overlap" ""; do timeout -k 10 600 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-extras $o > gpurun_out/b.log 2>&1 || (tail -20 gpurun_out/b.log; exit 1); python3 -c "import json,sys; d=json.loads(open('gpurun_out/b.log').read().strip().splitlines()[-1]); print('overlap=$o', round(d['value'],2), round(d['ms_per_step'],1))"; done
