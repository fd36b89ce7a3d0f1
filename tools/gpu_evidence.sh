#!/bin/bash
# End-of-round evidence on HEAD (run under gpurun from the repo root): the GPU suite + smoke +
# default bench (tools/gpu_suite.sh), the per-launch table, rocprofv3 kernel stats and the PMC
# FETCH_SIZE / WRITE_SIZE passes (tools/profile_round.sh).  Copy the results you cite from
# gpurun_out/ into profiles/.   usage: tools/gpu_evidence.sh TAG
set -u
tag=${1:?usage: tools/gpu_evidence.sh TAG}
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_suite.sh "$tag" || exit 1
timeout -k 10 200 python -u tools/launch_table.py --top 50 > gpurun_out/${tag}_launch_table.txt 2>&1 || { echo "launch table failed"; exit 94; }
head -12 gpurun_out/${tag}_launch_table.txt
bash tools/profile_round.sh ${tag}_p 10 || exit 1
