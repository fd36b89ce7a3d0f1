# round-6: config 5 -- the pair row-tile rule and the partial-round conv rule each on their own (3 streams)
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
step() { local name=$1 secs=$2; shift 2; timeout -k 10 "$secs" "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc $(grep -o '"value":[0-9.]*' gpurun_out/$name.log | head -1)"; if [ $rc -gt 1 ]; then exit $rc; fi; }
w="--no-train --no-cpu-baseline --no-config3 --no-config5 --steps 20 --warmup 5"
for r in 1 2; do
  step r06ac_c5pair_$r 240 python -u bench.py $w --workload config5 --gemm-flags 524288
  step r06ac_c5conv_$r 240 python -u bench.py $w --workload config5 --ffn-knob 256
  step r06ac_c5old_$r 240 python -u bench.py $w --workload config5 --ffn-knob 256 --gemm-flags 524288
  step r06ac_c5s1new_$r 240 python -u bench.py $w --workload config5 --streams 1
  step r06ac_c5s1old_$r 240 python -u bench.py $w --workload config5 --streams 1 --ffn-knob 256 --gemm-flags 524288
done
