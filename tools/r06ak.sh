# round-6: N = 128 3x3 convs (stage 2) after the gemm_dma read-ahead change: which tile now wins
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
sh="28,100,167,128,128,3,1;28,200,334,128,128,3,2;12,100,167,128,128,3,1;4,135,240,128,128,3,1"
timeout -k 10 300 python -u tools/conv_ab.py --iters 30 --shapes "$sh" > gpurun_out/r06ak_conv.log 2>&1 || { tail -20 gpurun_out/r06ak_conv.log; exit 9; }
timeout -k 10 300 python -u tools/conv_ab.py --iters 30 --shapes "$sh" >> gpurun_out/r06ak_conv.log 2>&1 || { tail -20 gpurun_out/r06ak_conv.log; exit 9; }
grep -v amdgpu gpurun_out/r06ak_conv.log
