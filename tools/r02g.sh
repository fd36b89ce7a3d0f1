set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_msda_gpu.py -x -q --timeout 120 --timeout-method thread -k "encoder" 2>&1 | tail -3 || exit 1
for b in 8 16; do
  timeout -k 10 120 python tools/bench_msda.py --batch $b --order || exit 1
  timeout -k 10 120 python tools/bench_msda.py --batch $b --enc || exit 1
  timeout -k 10 120 python tools/bench_msda.py --batch $b --enc --noise 1.0 || exit 1
done
