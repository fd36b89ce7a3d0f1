# round-6: fused FFN with the last partial round on 128-row tiles (ffn knob 32) vs default, config 2 (+ bit-identity probe)
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
step() { local name=$1 secs=$2; shift 2; timeout -k 10 "$secs" "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc $(grep -o '"value":[0-9.]*' gpurun_out/$name.log | head -1) $(grep -o '"ffn":{[^}]*}' gpurun_out/$name.log | head -1)"; if [ $rc -gt 1 ]; then exit $rc; fi; }
step r06o_ident 200 python -u tools/ffn_split_probe.py
cat gpurun_out/r06o_ident.log | tail -4
q="--no-train --no-config3 --no-config5 --no-cpu-baseline --steps 20 --warmup 5"
for r in 1 2 3; do
  step r06o_k0_$r 240 python -u bench.py $q
  step r06o_k32_$r 240 python -u bench.py $q --ffn-knob 32
done
