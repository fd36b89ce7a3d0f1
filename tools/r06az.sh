# round-6: config-2 in-flight batch on the final kernels: 28 (default) vs 24 vs 32, interleaved
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
step() { local name=$1 secs=$2; shift 2; timeout -k 10 "$secs" "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc $(grep -o '"value":[0-9.]*' gpurun_out/$name.log | head -1)"; if [ $rc -gt 1 ]; then exit $rc; fi; }
w="--no-train --no-cpu-baseline --no-config3 --no-config5 --steps 20 --warmup 5"
for r in 1 2; do
  step r06az_b28_$r 240 python -u bench.py $w
  step r06az_b24_$r 240 python -u bench.py $w --batch 24
  step r06az_b32_$r 240 python -u bench.py $w --batch 32
done
