# round-6: + residual GEMMs with N > 256 on 8-wave 512-column groups (in-tree) vs the previous library
# (tools/ab/libkinet_base.so = b7938cf) -- tests, launch-table rows, interleaved bench
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_gpu.py \
  -k "group_variants or rw_gemm or rw_conv1x1 or conv2d_nhwc or backbone" > gpurun_out/r06ap_tests.log 2>&1 || { tail -30 gpurun_out/r06ap_tests.log; exit 9; }
tail -2 gpurun_out/r06ap_tests.log
for lib in kinet_amd/_lib/libkinet_amd.so tools/ab/libkinet_base.so; do
  KINET_AMD_LIB=$lib timeout -k 10 200 python -u tools/launch_table.py --workload config2 --top 60 > gpurun_out/r06ap_lt2.log 2>&1 || exit 9
  echo "$lib: $(grep -h ', 128, 512, 1, 1)\|, 256, 1024, 1, 1)\|total' gpurun_out/r06ap_lt2.log | tr '\n' '|')"
done
step() { local name=$1 secs=$2; shift 2; timeout -k 10 "$secs" "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc $(grep -o '"value":[0-9.]*' gpurun_out/$name.log | head -1)"; if [ $rc -gt 1 ]; then exit $rc; fi; }
w="--no-train --no-cpu-baseline --no-config3 --no-config5 --steps 20 --warmup 5"
for r in 1 2; do
  step r06ap_new_$r 240 python -u bench.py $w
  KINET_AMD_LIB=tools/ab/libkinet_base.so step r06ap_old_$r 240 python -u bench.py $w
done
