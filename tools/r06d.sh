# round-6 A/B: bottleneck pairs at all widths on configs 3 and 5 (interleaved on one box)
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
step() { local name=$1 secs=$2; shift 2; timeout -k 10 "$secs" "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -o '"value": *[0-9.]*' gpurun_out/$name.log | head -1; if [ $rc -ne 0 ]; then tail -5 gpurun_out/$name.log; exit $rc; fi; }
c3="--workload config3 --no-train --no-cpu-baseline --steps 8 --warmup 2"
c5="--workload config5 --no-train --no-cpu-baseline --steps 8 --warmup 2"
for r in 1 2; do
  step r06d_c3pw64_$r 300 python -u bench.py $c3 --pair-widths 64 --detail gpurun_out/r06d_c3pw64_$r.json
  step r06d_c3pwall_$r 300 python -u bench.py $c3 --pair-widths 64,128,256 --detail gpurun_out/r06d_c3pwall_$r.json
  step r06d_c3pw256_$r 300 python -u bench.py $c3 --pair-widths 64,256 --detail gpurun_out/r06d_c3pw256_$r.json
  step r06d_c5pw64_$r 300 python -u bench.py $c5 --pair-widths 64 --detail gpurun_out/r06d_c5pw64_$r.json
  step r06d_c5pwall_$r 300 python -u bench.py $c5 --pair-widths 64,128,256 --detail gpurun_out/r06d_c5pwall_$r.json
  step r06d_c5pw128_$r 300 python -u bench.py $c5 --pair-widths 64,128 --detail gpurun_out/r06d_c5pw128_$r.json
done
