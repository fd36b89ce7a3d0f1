# config-2 bench at several --batch values (3 streams), interleaved: frames/s per batch
set -e
mkdir -p gpurun_out
for rep in 1 2; do
for b in ${BATCHES:-16 24 32 12}; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-train --no-config3 --no-config5 --batch $b > gpurun_out/ab_batch_$b.log 2>&1
  echo "batch=$b $(grep -o '"value": [0-9.]*' gpurun_out/ab_batch_$b.log | head -1)"
done
done
