# round-6: HEAD vs 9685f37's library on one box (is the r06av gate's 1362 the box or the code?)
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
step() { local name=$1 secs=$2; shift 2; timeout -k 10 "$secs" "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc $(grep -o '"value":[0-9.]*' gpurun_out/$name.log | head -1)"; if [ $rc -gt 1 ]; then exit $rc; fi; }
w="--no-train --no-cpu-baseline --no-config3 --no-config5 --steps 20 --warmup 5"
for r in 1 2; do
  step r06aw_head_$r 240 python -u bench.py $w
  KINET_AMD_LIB=tools/ab/libkinet_base.so step r06aw_base_$r 240 python -u bench.py $w
done
