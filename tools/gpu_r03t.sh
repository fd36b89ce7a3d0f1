# round-3 A/B + train check (run from the repo root under gpurun)
mkdir -p gpurun_out && export TMPDIR=/tmp && \
timeout -k 10 120 python tools/ffn_probe.py --rows 355568 --iters 10 > gpurun_out/r03t_ffn_probe.log 2>&1 && \
timeout -k 10 120 python tools/ffn_probe.py --rows 177784 --iters 10 >> gpurun_out/r03t_ffn_probe.log 2>&1 && \
timeout -k 10 300 python -u -m pytest tests/test_autograd_gpu.py tests/test_train_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03t_gputest.log 2>&1 && \
timeout -k 10 300 python tools/bench_train.py --steps 5 --warmup 2 > gpurun_out/r03t_train.json 2> gpurun_out/r03t_train.err && \
rm -rf gpurun_out/prof_r03t && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r03t -o run -- python tools/bench_train.py --steps 3 --warmup 1 > gpurun_out/r03t_trainprof.log 2>&1 && \
cp gpurun_out/prof_r03t/run_kernel_stats.csv gpurun_out/r03t_train_kernel_stats.csv && rm -rf gpurun_out/prof_r03t
