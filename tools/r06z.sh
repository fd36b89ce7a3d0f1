# round-6: HIP stream priorities of the three in-flight slots (config 2), one box
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
python -c "import torch; print('priority range', torch.cuda.Stream.priority_range())"
step() { local name=$1 secs=$2; shift 2; timeout -k 10 "$secs" "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc $(grep -o '"value":[0-9.]*' gpurun_out/$name.log | head -1)"; tail -1 gpurun_out/$name.log | cut -c1-120; if [ $rc -gt 1 ]; then exit $rc; fi; }
q="--no-train --no-config3 --no-config5 --no-cpu-baseline --steps 20 --warmup 5"
for r in 1 2; do
  step r06z_p000_$r 240 python -u bench.py $q
  step r06z_p100_$r 240 python -u bench.py $q --stream-prio=-1,0,0
  step r06z_p210_$r 240 python -u bench.py $q --stream-prio=-2,-1,0
done
