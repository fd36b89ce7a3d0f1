# round-4: records epilogue v2 (branch-free, permlane reductions) + bench A/B matrix
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/rec_ab.py > gpurun_out/r04d_rec_ab.log 2>&1 || exit 97
cat gpurun_out/r04d_rec_ab.log
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -k "records" > gpurun_out/r04d_new.log 2>&1; rc=$?; tail -6 gpurun_out/r04d_new.log; case $rc in 0|1) ;; *) exit 99;; esac
for v in "rec1:--msda-records 1" "rec0:--msda-records 0" "rec1g2:--msda-records 1 --gemm-flags 2" "rec0g2:--msda-records 0 --gemm-flags 2" "rec1f8:--msda-records 1 --ffn-knob 8"; do
  n=${v%%:*}; args=${v#*:}
  timeout -k 10 240 python -u bench.py --steps 30 --warmup 5 --no-train --no-config5 --no-cpu-baseline $args > gpurun_out/r04d_ab_$n.log 2>&1 || exit 95
  python - "$n" gpurun_out/r04d_ab_$n.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[2]) if l.startswith('{')][0])
r = d['roofline']
print(f"[{sys.argv[1]}] {d['value']:.1f} frames/s  enc {r['encoder_launch']['ms']*1e3:.1f} us  frac {r['frac']:.3f}  kxk {d['roofline_gemm_conv_split'].get('conv_kxk', {}).get('frac', 0):.3f}  fam {d['device_ms_per_step_by_family']}")
PY
done
