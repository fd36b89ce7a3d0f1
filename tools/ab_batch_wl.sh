# usage: WL=config3 BATCHES="8 12 16" bash tools/ab_batch_wl.sh: interleaved --batch sweep of one workload
set -e
mkdir -p gpurun_out
for rep in 1 2; do
for b in $BATCHES; do
  timeout -k 10 300 python -u bench.py --workload $WL --no-cpu-baseline --batch $b > gpurun_out/ab_${WL}_b$b.log 2>&1
  echo "$WL batch=$b $(grep -o '"value": [0-9.]*' gpurun_out/ab_${WL}_b$b.log | head -1)"
done
done
