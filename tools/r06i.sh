# round-6: records GEMM ring depth after the drain fix: 3 WGs x 2 slots (default) vs 2 WGs x 4 / x 3 slots
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
step() { local name=$1 secs=$2; shift 2; timeout -k 10 "$secs" "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -o '"value":[0-9.]*\|"encoder_call":{[^}]*}' gpurun_out/$name.log | head -3 | cut -c1-120 | tr '\n' ' '; echo; tail -1 gpurun_out/$name.log | cut -c1-200; if [ $rc -gt 1 ]; then exit $rc; fi; }
step r06i_test 600 python -u -m pytest tests/test_msda_gpu.py tests/test_model_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "record or frame_shared or shared_frame"
q="--no-train --no-config3 --no-config5 --no-cpu-baseline --steps 20 --warmup 5"
for r in 1 2; do
  step r06i_f0_$r 300 python -u bench.py $q --detail gpurun_out/r06i_f0_$r.json
  step r06i_f8192_$r 300 python -u bench.py $q --gemm-flags 8192 --detail gpurun_out/r06i_f8192_$r.json
  step r06i_f16384_$r 300 python -u bench.py $q --gemm-flags 16384 --detail gpurun_out/r06i_f16384_$r.json
done
