# round-6: records GEMM without the per-tile DMA drain -- tests, then bench A/B vs the previous library
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
step() { local name=$1 secs=$2; shift 2; timeout -k 10 "$secs" "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -o '"value":[0-9.]*\|"encoder_call":{[^}]*}' gpurun_out/$name.log | head -3 | cut -c1-200 | tr '\n' ' '; echo; tail -2 gpurun_out/$name.log | cut -c1-200; if [ $rc -gt 1 ]; then exit $rc; fi; }
step r06h_test 600 python -u -m pytest tests/test_msda_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "record or frame_shared"
q="--no-train --no-config3 --no-config5 --no-cpu-baseline --steps 20 --warmup 5"
for r in 1 2; do
  step r06h_new_$r 300 python -u bench.py $q --detail gpurun_out/r06h_new_$r.json
  KINET_AMD_LIB=tools/ab/libkinet_base.so step r06h_base_$r 300 python -u bench.py $q --detail gpurun_out/r06h_base_$r.json
done
