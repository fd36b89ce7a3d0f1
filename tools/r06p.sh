# round-6: decoder-sized GEMMs (M = 8400 at batch 28) on the tiled kernels instead of the resident-weight one (gemm flag 16384)
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
step() { local name=$1 secs=$2; shift 2; timeout -k 10 "$secs" "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc $(grep -o '"value":[0-9.]*' gpurun_out/$name.log | head -1)"; if [ $rc -gt 1 ]; then exit $rc; fi; }
q="--no-train --no-config3 --no-config5 --no-cpu-baseline --steps 20 --warmup 5"
for r in 1 2 3; do
  step r06p_f0_$r 240 python -u bench.py $q
  step r06p_f16384_$r 240 python -u bench.py $q --gemm-flags 16384
done
step r06p_lt 300 python -u tools/launch_table.py --workload config2 --top 60
step r06p_lt16384 300 python -u tools/launch_table.py --workload config2 --top 60 --gemm-flags 16384
