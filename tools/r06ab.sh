# round-6: shape-adaptive pair row tiles + partial-round conv tiles (config 5 stage 3) -- tests + bench A/B
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gemm_gpu.py \
  -k "pair or full_rounds or partial_round or big_conv" > gpurun_out/r06ab_tests.log 2>&1 || { tail -30 gpurun_out/r06ab_tests.log; exit 9; }
tail -3 gpurun_out/r06ab_tests.log
step() { local name=$1 secs=$2; shift 2; timeout -k 10 "$secs" "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc $(grep -o '"value":[0-9.]*' gpurun_out/$name.log | head -1)"; if [ $rc -gt 1 ]; then exit $rc; fi; }
w="--no-train --no-cpu-baseline --no-config3 --no-config5 --steps 20 --warmup 5"
for r in 1 2; do
  step r06ab_c5new_$r 240 python -u bench.py $w --workload config5
  step r06ab_c5old_$r 240 python -u bench.py $w --workload config5 --ffn-knob 256 --gemm-flags 524288
done
step r06ab_c3new 240 python -u bench.py $w --workload config3
step r06ab_c2new 240 python -u bench.py $w --workload config2
