# usage: WL=config2 STREAMS="3 4" bash tools/ab_streams.sh: interleaved --streams sweep at the default batch
set -e
mkdir -p gpurun_out
for rep in 1 2; do
for s in $STREAMS; do
  timeout -k 10 300 python -u bench.py --workload $WL --no-cpu-baseline --no-train --no-config3 --no-config5 --streams $s > gpurun_out/ab_${WL}_s$s.log 2>&1
  echo "$WL streams=$s $(grep -o '"value": [0-9.]*' gpurun_out/ab_${WL}_s$s.log | head -1)"
done
done
