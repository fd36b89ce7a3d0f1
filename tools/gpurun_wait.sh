#!/bin/bash
# Submit one gpurun command, re-submitting ONLY while the pool reports no free box / slot
# (nothing ran, nothing charged: exit 3, or a "transient" status); any other outcome -- the
# command ran, failed, timed out or was refused -- ends the loop.  Never retries a GPU run.
#   usage: tools/gpurun_wait.sh LOG TIMEOUT 'command' [max_attempts]
log=$1; to=$2; cmd=$3; max=${4:-12}
for i in $(seq 1 "$max"); do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$cmd" > "$log" 2>&1
  rc=$?
  if [ $rc -eq 3 ] || grep -q 'status=transient' "$log"; then
    echo "[gpurun_wait] attempt $i: no box ($rc), waiting" >> "$log.attempts"
    sleep 150
    continue
  fi
  echo "[gpurun_wait] attempt $i: rc=$rc" >> "$log.attempts"
  exit $rc
done
exit 3
