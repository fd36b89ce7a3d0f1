# round-6: 8-wave single column group for the x + pos projections (records GEMM, K = 288 A2 GEMMs) --
# tests, then interleaved bench A/B vs flag 268435456 (the 4-wave 192-column groups) on configs 3, 5, 2
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_gpu.py tests/test_msda_gpu.py \
  -k "rw288 or records or group_variants" > gpurun_out/r06an_tests.log 2>&1 || { tail -30 gpurun_out/r06an_tests.log; exit 9; }
tail -2 gpurun_out/r06an_tests.log
for f in 0 268435456; do
  timeout -k 10 200 python -u tools/launch_table.py --workload config3 --gemm-flags $f --top 8 > gpurun_out/r06an_lt3_$f.log 2>&1 || exit 9
  echo "config3 flags $f: $(grep -h 'headmajor_ex\|total' gpurun_out/r06an_lt3_$f.log | tr '\n' '|')"
done
step() { local name=$1 secs=$2; shift 2; timeout -k 10 "$secs" "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc $(grep -o '"value":[0-9.]*' gpurun_out/$name.log | head -1) $(grep -o '"encoder_call":{[^}]*}' gpurun_out/$name.log | head -1)"; if [ $rc -gt 1 ]; then exit $rc; fi; }
w="--no-train --no-cpu-baseline --no-config3 --no-config5 --steps 20 --warmup 5"
for r in 1 2; do
  step r06an_c3new_$r 240 python -u bench.py $w --workload config3
  step r06an_c3old_$r 240 python -u bench.py $w --workload config3 --gemm-flags 268435456
  step r06an_c5new_$r 240 python -u bench.py $w --workload config5
  step r06an_c5old_$r 240 python -u bench.py $w --workload config5 --gemm-flags 268435456
  step r06an_c2new_$r 240 python -u bench.py $w
  step r06an_c2old_$r 240 python -u bench.py $w --gemm-flags 268435456
done
