#!/bin/bash
# gpurun, retried only while the pool has no free box (exit code 3: nothing ran, nothing charged);
# any other outcome (including a failed or timed-out command) is returned as is.
#   tools/gpurun_wait.sh TIMEOUT 'command' LOG
T=$1; CMD=$2; LOG=$3
for i in $(seq 1 12); do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$CMD" > "$LOG" 2>&1
  rc=$?
  if [ $rc -ne 3 ] && ! grep -q "status=transient" "$LOG"; then exit $rc; fi
  echo "[gpurun_wait] no box (try $i), retrying in 180 s" >> "$LOG.wait"
  sleep 180
done
exit 3
