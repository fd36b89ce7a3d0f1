set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_msda_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r02d_msda_tests.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/r02d_msda_tests.log; exit 1; }
tail -2 gpurun_out/r02d_msda_tests.log
for b in 8 16; do
  timeout -k 10 120 python tools/bench_msda.py --batch $b --order >> gpurun_out/r02d_bench_msda.log 2>&1 || exit 1
  timeout -k 10 120 python tools/bench_msda.py --batch $b --enc >> gpurun_out/r02d_bench_msda.log 2>&1 || exit 1
  timeout -k 10 120 python tools/bench_msda.py --batch $b --enc --noise 1.0 >> gpurun_out/r02d_bench_msda.log 2>&1 || exit 1
  timeout -k 10 120 python tools/bench_msda.py --batch $b --order --noise 1.0 >> gpurun_out/r02d_bench_msda.log 2>&1 || exit 1
done
cat gpurun_out/r02d_bench_msda.log | grep msda
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r02d_bench.log 2>&1 || exit 1
tail -1 gpurun_out/r02d_bench.log | cut -c1-400
