# round-6: GPU suite on the pair-width default, batch / stream sweep for config 2, launch tables
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
step() { local name=$1 secs=$2; shift 2; timeout -k 10 "$secs" "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -o '"value": *[0-9.]*' gpurun_out/$name.log | head -1; tail -2 gpurun_out/$name.log | cut -c1-200; if [ $rc -gt 1 ]; then exit $rc; fi; }
step r06e_gputest 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -s -k "fullsize or model or bottleneck or pair or shared"
q="--no-train --no-config3 --no-config5 --no-cpu-baseline --steps 20 --warmup 5"
for r in 1 2; do
  step r06e_b24_$r 240 python -u bench.py $q --detail gpurun_out/r06e_b24_$r.json
  step r06e_b32_$r 240 python -u bench.py $q --batch 32 --detail gpurun_out/r06e_b32_$r.json
  step r06e_b28_$r 240 python -u bench.py $q --batch 28 --detail gpurun_out/r06e_b28_$r.json
  step r06e_b24s4_$r 240 python -u bench.py $q --streams 4 --detail gpurun_out/r06e_b24s4_$r.json
done
step r06e_lt2 300 python -u tools/launch_table.py --workload config2 --top 60
step r06e_lt3 300 python -u tools/launch_table.py --workload config3 --top 40
step r06e_lt5 300 python -u tools/launch_table.py --workload config5 --top 40
