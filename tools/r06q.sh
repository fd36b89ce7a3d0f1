# round-6: D = 128 bottleneck pair with 3 row tiles per wave (ffn knob 64) vs 2 -- bit identity, bench A/B, launch tables
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
step() { local name=$1 secs=$2; shift 2; timeout -k 10 "$secs" "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc $(grep -o '"value":[0-9.]*' gpurun_out/$name.log | head -1)"; tail -1 gpurun_out/$name.log | cut -c1-120; if [ $rc -gt 1 ]; then exit $rc; fi; }
step r06q_test 300 python -u -m pytest tests/test_gemm_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "pair"
q="--no-train --no-config3 --no-config5 --no-cpu-baseline --steps 20 --warmup 5"
for r in 1 2 3; do
  step r06q_k0_$r 240 python -u bench.py $q
  step r06q_k64_$r 240 python -u bench.py $q --ffn-knob 64
done
step r06q_lt 300 python -u tools/launch_table.py --workload config2 --top 40
step r06q_lt64 300 python -u tools/launch_table.py --workload config2 --top 40 --ffn-knob 64
