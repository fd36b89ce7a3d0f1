# round-6: encoder sampler cache policy of the streamed operands (A/B, config 2 + config 5, one box)
#   base: default; st16: output stores sc1 (drop the line from L2); st16ld2: + records loads nt; st2: stores nt
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
step() { local name=$1 secs=$2; shift 2; timeout -k 10 "$secs" "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc $(grep -o '"value":[0-9.]*' gpurun_out/$name.log | head -3 | tr '\n' ' ') $(grep -o '"avg_launch_ms":[0-9.]*' gpurun_out/$name.log | head -1) $(grep -o '"traffic_x_algorithmic":[0-9.]*' gpurun_out/$name.log | head -1)"; if [ $rc -gt 1 ]; then exit $rc; fi; }
q="--no-train --no-config3 --no-cpu-baseline --steps 20 --warmup 5"
for r in 1 2; do
  for v in base st16 st16ld2 st2; do
    KINET_AMD_LIB=tools/ab/libkinet_$v.so step r06l_${v}_$r 300 python -u bench.py $q
  done
done
for v in base st16 st16ld2; do
  KINET_AMD_LIB=tools/ab/libkinet_$v.so step r06l_enc_$v 200 python -u tools/bench_msda.py --rec --order --batch 28 --iters 40
done
