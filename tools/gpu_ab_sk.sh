for v in "GANAMD_RESNET_BRANCHES=0 GANAMD_SK_BRANCHES=1" "GANAMD_RESNET_BRANCHES=1 GANAMD_SK_BRANCHES=0"; do
  env $v timeout -k 10 600 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-extras > gpurun_out/b.log 2>&1
  echo "$v rc=$?"; python3 -c "import json; d=json.loads(open('gpurun_out/b.log').read().strip().splitlines()[-1]); print(round(d['value'],2), round(d['ms_per_step'],1))" || tail -3 gpurun_out/b.log
done
