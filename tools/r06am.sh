# round-6: records GEMM (kinet_msda_sample_records) as ONE 8-wave 384-column group per row tile (x + pos read
# once per tile) vs the default two 4-wave 192-column groups sharing it through L2: flag 268435456 = 8 waves
# one per CU, 536870912 = 8 waves two per CU
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
for f in 0 268435456 536870912; do
  timeout -k 10 120 python -c "import sys; sys.path.insert(0, '.'); from kinet_amd import _native; _native.lib().kinet_gemm_set_flags($f); import runpy; runpy.run_path('tools/enc_sig_probe.py', run_name='__main__')" 2>&1 | grep -v amdgpu | sed "s/^/flags $f: /" || exit 9
done
for r in 1 2; do
  for f in 0 268435456 536870912; do
    timeout -k 10 200 python -u tools/launch_table.py --workload config2 --gemm-flags $f --filter sample_records > gpurun_out/r06am_lt_${f}_$r.log 2>&1 || { tail gpurun_out/r06am_lt_${f}_$r.log; exit 9; }
    echo "flags $f rep $r: $(grep -h sample_records gpurun_out/r06am_lt_${f}_$r.log | head -1)"
  done
done
step() { local name=$1 secs=$2; shift 2; timeout -k 10 "$secs" "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc $(grep -o '"value":[0-9.]*' gpurun_out/$name.log | head -1) $(grep -o '"encoder_call":{[^}]*}' gpurun_out/$name.log | head -1)"; if [ $rc -gt 1 ]; then exit $rc; fi; }
w="--no-train --no-cpu-baseline --no-config3 --no-config5 --steps 20 --warmup 5"
for r in 1 2; do
  step r06am_b0_$r 240 python -u bench.py $w
  step r06am_b1_$r 240 python -u bench.py $w --gemm-flags 268435456
  step r06am_b2_$r 240 python -u bench.py $w --gemm-flags 536870912
done
