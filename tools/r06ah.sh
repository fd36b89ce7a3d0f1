# round-6: FFN read-ahead schedule as the default -- FFN / encoder GPU tests + config-2 bench
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/ -m gpu \
  -k "ffn or encoder_layer or detr_config2 or transformer" > gpurun_out/r06ah_tests.log 2>&1 || { tail -30 gpurun_out/r06ah_tests.log; exit 9; }
tail -3 gpurun_out/r06ah_tests.log
timeout -k 10 120 python -u tools/ffn_probe.py --rows 622244 --iters 30 --knobs 0,0,0 2>&1 | grep -v amdgpu
step() { local name=$1 secs=$2; shift 2; timeout -k 10 "$secs" "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc $(grep -o '"value":[0-9.]*' gpurun_out/$name.log | head -1) $(grep -o '"ffn":{[^}]*}' gpurun_out/$name.log | head -1)"; if [ $rc -gt 1 ]; then exit $rc; fi; }
w="--no-train --no-cpu-baseline --no-config3 --no-config5 --steps 20 --warmup 5"
step r06ah_c2_1 240 python -u bench.py $w
step r06ah_c2_2 240 python -u bench.py $w
