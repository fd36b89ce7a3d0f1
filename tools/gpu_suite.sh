#!/bin/bash
# The GPU gate of one change (run from the repo root under gpurun): the -m gpu suite, smoke(),
# then the default bench line.  Each step under its own time limit; the first crash / timeout /
# failure ends the script.  Logs: gpurun_out/<tag>_{gputest,smoke,bench}.log, the bench JSON
# line in gpurun_out/<tag>_bench.json.
# usage: tools/gpu_suite.sh TAG [pytest -k expression] [bench args...]
set -u
tag=$1; kexpr=${2:-}; shift; [ $# -gt 0 ] && shift
export TMPDIR=/tmp
mkdir -p gpurun_out
run() { local secs=$1 log=$2; shift 2; timeout -k 10 "$secs" "$@" > "$log" 2>&1; local rc=$?; tail -4 "$log";
        if [ $rc -ne 0 ]; then echo "[gpu_suite] rc=$rc: $*"; exit 99; fi; }
if [ -n "$kexpr" ]; then
  run 900 gpurun_out/${tag}_gputest.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$kexpr"
else
  run 900 gpurun_out/${tag}_gputest.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
fi
run 300 gpurun_out/${tag}_smoke.log python -c "import __graft_entry__ as g; g.smoke()"
run 600 gpurun_out/${tag}_bench.log python -u bench.py "$@"
grep '^{' gpurun_out/${tag}_bench.log > gpurun_out/${tag}_bench.json
echo "[gpu_suite] done $tag"
