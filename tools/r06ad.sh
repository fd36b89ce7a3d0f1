# round-6: solo-launch policy (kinet_set_solo_launch) -- tests + config 5 on 3 streams (throughput) and 1 stream (solo)
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gemm_gpu.py \
  -k "pair or full_rounds or partial_round or big_conv" > gpurun_out/r06ad_tests.log 2>&1 || { tail -30 gpurun_out/r06ad_tests.log; exit 9; }
tail -3 gpurun_out/r06ad_tests.log
step() { local name=$1 secs=$2; shift 2; timeout -k 10 "$secs" "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc $(grep -o '"value":[0-9.]*' gpurun_out/$name.log | head -1)"; if [ $rc -gt 1 ]; then exit $rc; fi; }
w="--no-train --no-cpu-baseline --no-config3 --no-config5 --steps 20 --warmup 5"
for r in 1 2; do
  step r06ad_c5s3_$r 240 python -u bench.py $w --workload config5
  step r06ad_c5s1_$r 240 python -u bench.py $w --workload config5 --streams 1
  step r06ad_c5s1rt2_$r 240 python -u bench.py $w --workload config5 --streams 1 --ffn-knob 256
done
