# round-6: 32-column head-major stores through an LDS transpose (default) vs direct 16-byte unit stores
# (flag 1073741824): tests, config-2 launch-table rows, interleaved bench
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_gpu.py tests/test_msda_gpu.py \
  -k "headmajor or rw_gemm or rw_row_tile or group_variants or encoder" > gpurun_out/r06au_tests.log 2>&1 || { tail -30 gpurun_out/r06au_tests.log; exit 9; }
tail -2 gpurun_out/r06au_tests.log
for f in 0 1073741824; do
  timeout -k 10 200 python -u tools/launch_table.py --workload config2 --gemm-flags $f --top 20 > gpurun_out/r06au_lt_$f.log 2>&1 || exit 9
  echo "config2 flags $f: $(grep -h 'headmajor\|total' gpurun_out/r06au_lt_$f.log | tr '\n' '|')"
done
step() { local name=$1 secs=$2; shift 2; timeout -k 10 "$secs" "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc $(grep -o '"value":[0-9.]*' gpurun_out/$name.log | head -1)"; if [ $rc -gt 1 ]; then exit $rc; fi; }
w="--no-train --no-cpu-baseline --no-config3 --no-config5 --steps 20 --warmup 5"
for r in 1 2; do
  step r06au_new_$r 240 python -u bench.py $w
  step r06au_old_$r 240 python -u bench.py $w --gemm-flags 1073741824
done
