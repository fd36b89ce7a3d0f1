#!/bin/bash
# Run one gpurun call, retrying only while the pool reports no free box (exit 3: nothing ran,
# nothing charged).  usage: tools/gpurun_retry.sh LOG TIMEOUT 'command'
log=$1; t=$2; cmd=$3
for i in $(seq 1 30); do
  /usr/local/graft/bin/gpurun --timeout "$t" -- "$cmd" > "$log" 2>&1
  rc=$?
  echo "[retry] attempt $i rc=$rc" >> "$log"
  [ $rc -ne 3 ] && exit $rc
  sleep 60
done
exit 3
