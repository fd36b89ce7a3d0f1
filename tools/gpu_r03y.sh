# strip encoder kernel A/B: branch-free per-point addresses (in-tree) vs the previous build (tools/ab/libenc_old.so)
mkdir -p gpurun_out && export TMPDIR=/tmp && \
timeout -k 10 180 python tools/enc_ab.py --batch 16 --iters 30 --reps 4 > gpurun_out/r03y_enc_ab.log 2>&1 && \
timeout -k 10 300 python -u -m pytest tests/test_msda_gpu.py tests/test_fullsize_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03y_gputest.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 15 --warmup 3 --no-train --no-cpu-baseline > gpurun_out/r03y_bench.log 2>&1
