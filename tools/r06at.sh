# round-6: K = 288 plain epilogues with 192 < N <= 384 (the d = 288 value projection, split head-major planes)
# on 8-wave 384-column groups (in-tree) vs the previous library (tools/ab/libkinet_base.so = 9685f37)
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_gpu.py tests/test_msda_gpu.py \
  -k "group_variants or rw288 or headmajor or split" > gpurun_out/r06at_tests.log 2>&1 || { tail -30 gpurun_out/r06at_tests.log; exit 9; }
tail -2 gpurun_out/r06at_tests.log
for lib in kinet_amd/_lib/libkinet_amd.so tools/ab/libkinet_base.so; do
  KINET_AMD_LIB=$lib timeout -k 10 200 python -u tools/launch_table.py --workload config3 --top 12 > gpurun_out/r06at_lt.log 2>&1 || exit 9
  echo "config3 $lib: $(grep -h 'split\|(266676, 288, 288)\|total' gpurun_out/r06at_lt.log | tr '\n' '|')"
done
step() { local name=$1 secs=$2; shift 2; timeout -k 10 "$secs" "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc $(grep -o '"value":[0-9.]*' gpurun_out/$name.log | head -1)"; if [ $rc -gt 1 ]; then exit $rc; fi; }
w="--no-train --no-cpu-baseline --no-config3 --no-config5 --steps 20 --warmup 5"
for r in 1 2; do
  step r06at_c3new_$r 240 python -u bench.py $w --workload config3
  KINET_AMD_LIB=tools/ab/libkinet_base.so step r06at_c3old_$r 240 python -u bench.py $w --workload config3
  step r06at_c5new_$r 240 python -u bench.py $w --workload config5
  KINET_AMD_LIB=tools/ab/libkinet_base.so step r06at_c5old_$r 240 python -u bench.py $w --workload config5
done
