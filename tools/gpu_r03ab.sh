# encoder A/B (first-flush widening + quad DPP reduce vs the previous build) + the whole GPU suite
mkdir -p gpurun_out && export TMPDIR=/tmp && \
timeout -k 10 180 python tools/enc_ab.py --batch 16 --iters 30 --reps 4 > gpurun_out/r03ab_enc_ab.log 2>&1 && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03ab_gputest.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 15 --warmup 3 --no-train --no-cpu-baseline > gpurun_out/r03ab_bench.log 2>&1
