# round-6: encoder MSDA call in frame chunks (records read back from the memory-side cache) -- identity, bench A/B
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
step() { local name=$1 secs=$2; shift 2; timeout -k 10 "$secs" "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc $(grep -o '"value":[0-9.]*' gpurun_out/$name.log | head -1) $(grep -o '"encoder_call":{[^}]*' gpurun_out/$name.log | head -1 | cut -c1-90)"; tail -2 gpurun_out/$name.log | cut -c1-150; if [ $rc -gt 1 ]; then exit $rc; fi; }
step r06w_ident 200 python -u tools/rec_chunk_probe.py
q="--no-train --no-config3 --no-config5 --no-cpu-baseline --steps 20 --warmup 5"
for r in 1 2; do
  step r06w_c0_$r 240 python -u bench.py $q
  step r06w_c7_$r 240 python -u bench.py $q --rec-chunk 7
  step r06w_c14_$r 240 python -u bench.py $q --rec-chunk 14
done
