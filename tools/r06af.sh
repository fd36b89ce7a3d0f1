# round-6: fused FFN, fragments read further ahead vs default (kinet_ffn_set_debug 4 = PF 1: A 2 / B 4 ahead,
# 512 = PF 2: A 2 / B 6, 1024 = PF 3: A 3 / B 4; PF >= 1 with the integer ReLU), batch-28 encoder FFN
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/ffn_probe.py --rows 622244 --iters 30 --knobs 0,0,4,512,1024,0,4,512,1024,0,4,512,1024 > gpurun_out/r06af_ffn.log 2>&1 || { cat gpurun_out/r06af_ffn.log; exit 9; }
grep -v amdgpu gpurun_out/r06af_ffn.log
timeout -k 10 120 python -u tools/ffn_probe.py --rows 622244 --iters 20 --knobs 0,4,512,1024 --dtype f16 2>&1 | grep -v amdgpu
timeout -k 10 120 python -u tools/ffn_probe.py --rows 88892 --iters 20 --knobs 0,4,512,1024 2>&1 | grep -v amdgpu
