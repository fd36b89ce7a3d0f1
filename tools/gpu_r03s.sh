mkdir -p gpurun_out && export TMPDIR=/tmp && \
timeout -k 10 300 python -u -m pytest tests/test_autograd_gpu.py tests/test_train_gpu.py tests/test_ddp_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03s_gputest.log 2>&1 && \
timeout -k 10 300 python tools/bench_train.py --steps 5 --warmup 2 > gpurun_out/r03s_train.json 2> gpurun_out/r03s_train.err && \
rm -rf gpurun_out/prof_r03s && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r03s -o run -- python tools/bench_train.py --steps 3 --warmup 1 > gpurun_out/r03s_trainprof.log 2>&1 && \
cp gpurun_out/prof_r03s/run_kernel_stats.csv gpurun_out/r03s_train_kernel_stats.csv && rm -rf gpurun_out/prof_r03s && \
timeout -k 10 300 python tools/launch_table.py --batch 16 --top 60 > gpurun_out/r03s_launch_table.txt 2>&1
