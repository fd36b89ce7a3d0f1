#!/bin/bash
# Run GPU steps in order under gpurun (from the repo root): each argument is
#   "NAME:SECONDS:COMMAND"
# and runs as `timeout -k 10 SECONDS bash -c COMMAND > gpurun_out/NAME.log 2>&1`.  A step that
# exits 0 or 1 (pytest: tests failed, nothing crashed) lets the next step run; any other status
# (a crash, an abort, a time limit: 2+, 124, 134, 137, 139, ...) ends the script there, so nothing
# else touches the GPU after a fault.  The tail of every log is printed.
#   usage: tools/gpu_steps.sh "diag:300:python -u tools/x.py" "tests:600:python -u -m pytest ..."
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
worst=0
for step in "$@"; do
  name=${step%%:*}; rest=${step#*:}; secs=${rest%%:*}; cmd=${rest#*:}
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "== $name rc=$rc"; tail -12 "gpurun_out/$name.log"
  [ $rc -gt $worst ] && worst=$rc
  if [ $rc -gt 1 ]; then echo "[gpu_steps] stopping after $name (rc=$rc)"; exit $rc; fi
done
exit $worst
