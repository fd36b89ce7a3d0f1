# round-6: 12-wave encoder sampler with two points' LDS corners in flight (KINET_ENC_WAVES=12) vs 16 waves
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
step() { local name=$1 secs=$2; shift 2; timeout -k 10 "$secs" "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc $(grep -o '"value":[0-9.]*' gpurun_out/$name.log | head -1) $(grep -o '"encoder_call":{[^}]*' gpurun_out/$name.log | head -1 | cut -c1-90)"; tail -1 gpurun_out/$name.log | cut -c1-150; if [ $rc -gt 1 ]; then exit $rc; fi; }
step r06y_sig16 200 python -u tools/enc_sig_probe.py
KINET_ENC_WAVES=12 step r06y_sig12 200 python -u tools/enc_sig_probe.py
KINET_ENC_WAVES=12 step r06y_test12 300 python -u -m pytest tests/test_msda_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "record or encoder or strip"
q="--no-train --no-config3 --no-config5 --no-cpu-baseline --steps 20 --warmup 5"
for r in 1 2; do
  step r06y_w16_$r 240 python -u bench.py $q
  KINET_ENC_WAVES=12 step r06y_w12_$r 240 python -u bench.py $q
done
