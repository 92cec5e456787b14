set -e
for b in 1 0 1 0; do GANAMD_BRANCHES=$b timeout -k 10 600 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-extras 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('branches=$b', round(d['value'],2), round(d['ms_per_step'],1))"; done
