# round-6: batch / streams sweep with graph replay on (the round-6 sweeps before the graph-check fix ran eager)
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
step() { local name=$1 secs=$2; shift 2; timeout -k 10 "$secs" "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc $(grep -o '"value":[0-9.]*' gpurun_out/$name.log | head -1) $(grep -o '"graph_check":"[^"]*"' gpurun_out/$name.log | head -1)"; if [ $rc -gt 1 ]; then exit $rc; fi; }
q="--no-train --no-config3 --no-config5 --no-cpu-baseline --steps 20 --warmup 5"
for r in 1 2; do
  step r06k_b28_$r 240 python -u bench.py $q
  step r06k_b24_$r 240 python -u bench.py $q --batch 24
  step r06k_b32_$r 240 python -u bench.py $q --batch 32
  step r06k_b28s4_$r 240 python -u bench.py $q --streams 4
  step r06k_b20s4_$r 240 python -u bench.py $q --batch 20 --streams 4
done
w="--no-train --no-cpu-baseline --no-config3 --no-config5 --steps 20 --warmup 5"
for r in 1 2; do
  step r06k_c3b12_$r 240 python -u bench.py $w --workload config3
  step r06k_c3b16_$r 240 python -u bench.py $w --workload config3 --batch 16
  step r06k_c3b8_$r 240 python -u bench.py $w --workload config3 --batch 8
  step r06k_c5b4_$r 240 python -u bench.py $w --workload config5
  step r06k_c5b6_$r 240 python -u bench.py $w --workload config5 --batch 6
done
