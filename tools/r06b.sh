set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
step() { local name=$1 secs=$2; shift 2; timeout -k 10 "$secs" "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -4 gpurun_out/$name.log; if [ $rc -gt 1 ]; then exit $rc; fi; }
step r06b_gputest 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step r06b_smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
for r in 1 2; do
  step r06b_enc_base_$r 120 python tools/bench_msda.py --rec --order --batch 24 --iters 40
  step r06b_enc_pf3_$r 120 env KINET_AMD_LIB=tools/ab/libkinet_pf3.so python tools/bench_msda.py --rec --order --batch 24 --iters 40
  step r06b_enc_pf6_$r 120 env KINET_AMD_LIB=tools/ab/libkinet_pf6.so python tools/bench_msda.py --rec --order --batch 24 --iters 40
done
