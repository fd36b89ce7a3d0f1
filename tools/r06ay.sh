# round-6: fused FFN with a 4-slot weight ring (kinet_ffn_set_debug 8192) vs the 3-slot default
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/ffn_probe.py --rows 622244 --iters 30 --knobs 0,0,8192,0,8192,0,8192 2>&1 | grep -v amdgpu
step() { local name=$1 secs=$2; shift 2; timeout -k 10 "$secs" "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc $(grep -o '"value":[0-9.]*' gpurun_out/$name.log | head -1) $(grep -o '"ffn":{[^}]*}' gpurun_out/$name.log | head -1)"; if [ $rc -gt 1 ]; then exit $rc; fi; }
w="--no-train --no-cpu-baseline --no-config3 --no-config5 --steps 20 --warmup 5"
for r in 1 2; do
  step r06ay_ns3_$r 240 python -u bench.py $w
  step r06ay_ns4_$r 240 python -u bench.py $w --ffn-knob 8192
done
