# round-6: config-5 layer-3/4 shapes (M = 32640 rows: half a round of 256-row tiles) -- conv tile variants, pair RT 1 vs 2
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/conv_ab.py --iters 20 --shapes "4,68,120,256,256,3,1;4,34,60,512,512,3,1;4,135,240,128,128,3,1;12,50,84,256,256,3,1" > gpurun_out/r06aa_conv.log 2>&1 || exit 9
grep -v amdgpu gpurun_out/r06aa_conv.log
timeout -k 10 300 python -u tools/launch_table.py --workload config5 --top 30 > gpurun_out/r06aa_lt5.log 2>&1 || exit 9
timeout -k 10 300 python -u tools/launch_table.py --workload config5 --top 30 --ffn-knob 128 > gpurun_out/r06aa_lt5_k128.log 2>&1 || exit 9
grep "bneck\|total" gpurun_out/r06aa_lt5.log gpurun_out/r06aa_lt5_k128.log
