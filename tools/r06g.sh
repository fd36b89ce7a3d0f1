# round-6: graph-replay check fixed -> graphed vs eager, config 2 / 3 / 5 (interleaved, one box)
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
step() { local name=$1 secs=$2; shift 2; timeout -k 10 "$secs" "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -o '"value":[0-9.]*\|"graph_check":"[^"]*"' gpurun_out/$name.log | head -4 | tr '\n' ' '; echo; grep '\[bench\]' gpurun_out/$name.log | head -3; if [ $rc -gt 1 ]; then exit $rc; fi; }
q="--no-train --no-cpu-baseline --steps 20 --warmup 5"
for r in 1 2; do
  step r06g_g1_$r 300 python -u bench.py $q --detail gpurun_out/r06g_g1_$r.json
  step r06g_g0_$r 300 python -u bench.py $q --graph 0 --detail gpurun_out/r06g_g0_$r.json
done
