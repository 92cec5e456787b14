#!/bin/bash
# r05n: memory stages of one B=64 graph-mode DP rank (overlap schedule)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
DP_MEMLOG=1 timeout -k 10 400 python3 -u -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr=127.0.0.1 \
  --master-port=29611 tests/dp_worker.py /tmp/r05n.pt graph overlap 64 > gpurun_out/r05n.log 2>&1
rc=$?
grep "\[mem\]" gpurun_out/r05n.log
exit $rc
