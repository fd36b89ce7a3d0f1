# round-6: compiler DMA drains removed (gemm_rw weights, pair t2 fragments, conv3x3 weights +
# staging writes) -- kernel tests, then bench A/B (configs 2 / 3 / 5) vs the previous library
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
step() { local name=$1 secs=$2; shift 2; timeout -k 10 "$secs" "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -o '"value":[0-9.]*' gpurun_out/$name.log | head -3 | tr '\n' ' '; echo; tail -1 gpurun_out/$name.log | cut -c1-150; if [ $rc -gt 1 ]; then exit $rc; fi; }
step r06j_test 600 python -u -m pytest tests/test_gemm_gpu.py tests/test_model_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "conv or pair or bottleneck or rw or resident or 288 or ffn"
q="--no-train --no-cpu-baseline --steps 20 --warmup 5"
for r in 1 2; do
  step r06j_new_$r 400 python -u bench.py $q --detail gpurun_out/r06j_new_$r.json
  KINET_AMD_LIB=tools/ab/libkinet_base.so step r06j_base_$r 400 python -u bench.py $q --detail gpurun_out/r06j_base_$r.json
done
step r06j_lt2 300 python -u tools/launch_table.py --workload config2 --top 40
KINET_AMD_LIB=tools/ab/libkinet_base.so step r06j_lt2base 300 python -u tools/launch_table.py --workload config2 --top 40
