#!/bin/bash
# round-4 k: full gate on HEAD (GPU suite, smoke, bench) + tracker / KineT throughput re-measure
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_suite.sh r04k || exit 1
timeout -k 10 300 python -u tools/track_hz.py > gpurun_out/r04k_track_hz.log 2>&1 || { echo "track_hz rc=$?"; tail -5 gpurun_out/r04k_track_hz.log; exit 1; }
tail -2 gpurun_out/r04k_track_hz.log
timeout -k 10 300 python -u tools/kinet_hz.py > gpurun_out/r04k_kinet_hz.log 2>&1 || { echo "kinet_hz rc=$?"; tail -5 gpurun_out/r04k_kinet_hz.log; exit 1; }
tail -2 gpurun_out/r04k_kinet_hz.log
