set -e
mkdir -p gpurun_out
for w in config3 config5; do
for f in 4194304 0 4194304 0; do
  timeout -k 10 300 python -u bench.py --workload $w --no-cpu-baseline --gemm-flags $f > gpurun_out/ab_${w}_$f.log 2>&1
  echo "$w flags=$f $(grep -o '"value": [0-9.]*' gpurun_out/ab_${w}_$f.log | head -1)"
done
done
