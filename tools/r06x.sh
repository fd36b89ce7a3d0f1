# round-6: in-flight batches for configs 3 / 5 with graph replay (default 3)
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
step() { local name=$1 secs=$2; shift 2; timeout -k 10 "$secs" "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc $(grep -o '"value":[0-9.]*' gpurun_out/$name.log | head -1)"; if [ $rc -gt 1 ]; then exit $rc; fi; }
w="--no-train --no-cpu-baseline --no-config3 --no-config5 --steps 20 --warmup 5"
for r in 1 2; do
  step r06x_c5s3_$r 240 python -u bench.py $w --workload config5
  step r06x_c5s4_$r 240 python -u bench.py $w --workload config5 --streams 4
  step r06x_c5s2b6_$r 240 python -u bench.py $w --workload config5 --streams 2 --batch 6
  step r06x_c3s3_$r 240 python -u bench.py $w --workload config3
  step r06x_c3s4b8_$r 240 python -u bench.py $w --workload config3 --streams 4 --batch 8
done
