set -e
for T in 256 512 1024 2048; do
  GANAMD_CONV_BLOCKS=$T timeout -k 10 300 python bench.py --no-cpu-baseline --steps 2 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print($T, d['value'], d['ms_per_step'])"
done
