# round-6: train leg with DDP find_unused_parameters True (reference) vs False, one box, interleaved
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
step() { local name=$1 secs=$2; shift 2; timeout -k 10 "$secs" "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc $(grep -o '"train":{[^}]*' gpurun_out/$name.log | grep -o '"value":[0-9.]*\|"s_per_step":[0-9.]*\|"host_glue_ms":[0-9.]*' | tr '\n' ' ')"; if [ $rc -gt 1 ]; then exit $rc; fi; }
q="--no-config3 --no-config5 --no-cpu-baseline --steps 4 --warmup 2 --train-steps 10"
for r in 1 2; do
  step r06s_fu1_$r 400 python -u bench.py $q --ddp-find-unused 1
  step r06s_fu0_$r 400 python -u bench.py $q --ddp-find-unused 0
done
