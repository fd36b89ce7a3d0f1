# round-6: LDS-DMA GEMM/conv kernel with the K-step's second-half fragments read during the first half
# (in-tree) vs the round-6 HEAD library (tools/ab/libkinet_base.so), conv shapes of configs 2 / 3 / 5
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
sh="28,50,84,256,256,3,1;28,25,42,512,512,3,1;28,100,167,256,256,3,2;28,50,84,512,512,3,2;12,50,84,256,256,3,1;4,34,60,512,512,3,1"
bash tools/ab_lib.sh tools/ab/libkinet_base.so python -u tools/conv_ab.py --iters 30 --shapes "$sh" > gpurun_out/r06ai_conv.log 2>&1 || { tail -20 gpurun_out/r06ai_conv.log; exit 9; }
grep "==\|heuristic\|t256x128\|t128x256\|dma4 " gpurun_out/r06ai_conv.log
