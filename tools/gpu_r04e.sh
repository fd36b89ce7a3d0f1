# round-4 gate on HEAD: the whole GPU suite, smoke, the per-launch table and the default bench line
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/launch_table.py --top 45 > gpurun_out/r04e_launch_table.txt 2>&1 || exit 94
head -30 gpurun_out/r04e_launch_table.txt
bash tools/gpu_suite.sh r04e
