#!/bin/bash
# Run one GPU step under its own time limit; stop the whole call on a crash/timeout
# (exit codes 124/137 timeout, 134 abort, 139 segfault) but continue after plain test
# failures.  usage: tools/gpu_step.sh SECONDS LOGFILE cmd...
secs=$1; log=$2; shift 2
timeout -k 10 "$secs" "$@" > "$log" 2>&1
rc=$?
echo "[gpu_step] rc=$rc cmd=$*" >> "$log"
tail -3 "$log"
case $rc in
  124|137|134|139|-6|-11) echo "[gpu_step] fatal rc=$rc, stopping"; exit 99;;
esac
exit 0
