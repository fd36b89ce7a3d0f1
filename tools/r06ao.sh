# round-6: K = 512, N = 256 GEMM (config-2 level-0 input projection) on one 8-wave 256-column group -- tests,
# launch-table row, bench A/B vs flag 268435456
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_gpu.py \
  -k "rw512 or rw_gemm or rw_matches or splitk_linear" > gpurun_out/r06ao_tests.log 2>&1 || { tail -30 gpurun_out/r06ao_tests.log; exit 9; }
tail -2 gpurun_out/r06ao_tests.log
for f in 0 268435456; do
  timeout -k 10 200 python -u tools/launch_table.py --workload config2 --gemm-flags $f --top 60 > gpurun_out/r06ao_lt2_$f.log 2>&1 || exit 9
  echo "config2 flags $f: $(grep -h ', 256, 512)\|total' gpurun_out/r06ao_lt2_$f.log | tr '\n' '|')"
done
step() { local name=$1 secs=$2; shift 2; timeout -k 10 "$secs" "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc $(grep -o '"value":[0-9.]*' gpurun_out/$name.log | head -1)"; if [ $rc -gt 1 ]; then exit $rc; fi; }
w="--no-train --no-cpu-baseline --no-config3 --no-config5 --steps 20 --warmup 5"
for r in 1 2; do
  step r06ao_c2new_$r 240 python -u bench.py $w
  step r06ao_c2old_$r 240 python -u bench.py $w --gemm-flags 268435456
done
