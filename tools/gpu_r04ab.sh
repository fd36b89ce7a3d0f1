#!/bin/bash
# round-4 ab: evidence on HEAD -- GPU suite + smoke + default bench, launch table, rocprofv3 stats + PMC passes
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_suite.sh r04ab || exit 1
timeout -k 10 200 python -u tools/launch_table.py --top 50 > gpurun_out/r04ab_launch_table.txt 2>&1 || { echo "launch table failed"; exit 94; }
head -12 gpurun_out/r04ab_launch_table.txt
bash tools/profile_round.sh r04ab_p 10 || exit 1
