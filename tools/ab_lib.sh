#!/bin/bash
# Headline bench (B = 64, default schedule) per library build: tools/ab_lib.sh TAG LIB.so [LIB2.so ...]
set -e
TAG=$1; shift
OUT=gpurun_out/${TAG}_ablib.txt
: > $OUT
for L in "$@"; do
  echo "== $L" >> $OUT
  GANAMD_SO=$(realpath $L) timeout -k 10 300 python3 bench.py --steps ${STEPS:-5} --warmup 1 --no-extras --no-cpu-baseline > gpurun_out/${TAG}_b.json 2> gpurun_out/${TAG}_b.log
  python3 -c "import json; d=json.loads(open('gpurun_out/${TAG}_b.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])" >> $OUT
done
cat $OUT
