#!/bin/bash
# A/B of the headline iteration's fake-batch schedule: pipelined side-stream fakes (default) vs
# all n_critic fakes from one segmented-BatchNorm generator forward, with and without the
# LDS-patch conv.  usage: tools/ab_fakes.sh TAG   (results in gpurun_out/TAG_ab.txt)
set -e
TAG=${1:-ab}
OUT=gpurun_out/${TAG}_ab.txt
: > $OUT
run() {
  echo "== $*" >> $OUT
  timeout -k 10 300 "$@" --steps ${STEPS:-5} --warmup 1 --no-extras --no-cpu-baseline > gpurun_out/${TAG}_b.json 2> gpurun_out/${TAG}_b.log
  grep "ms per phase" gpurun_out/${TAG}_b.log >> $OUT || true
  python3 -c "import json; d=json.loads(open('gpurun_out/${TAG}_b.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])" >> $OUT
}
run python3 bench.py
run python3 bench.py --fake-groups 1,4
run python3 bench.py --fake-groups 1,2,2
run python3 bench.py --fake-groups 4,1
run python3 bench.py --fake-groups 4,1 --overlap off
run python3 bench.py --fake-groups 2,3
cat $OUT
