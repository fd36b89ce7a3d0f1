# usage: bash tools/ab_flags.sh WORKLOAD FLAGS_A FLAGS_B [extra bench args]: A B A B bench runs
# (prints the line's value and, when present, the train sub-object's value)
set -e
w=$1; fa=$2; fb=$3; shift 3
mkdir -p gpurun_out
for f in $fa $fb $fa $fb; do
  timeout -k 10 300 python -u bench.py --workload $w --no-cpu-baseline --gemm-flags $f "$@" > gpurun_out/ab_${w}_$f.log 2>&1
  python - gpurun_out/ab_${w}_$f.log $w $f <<'PY'
import json, sys
line = [l for l in open(sys.argv[1]) if l.startswith('{')][-1]
d = json.loads(line)
t = (d.get('train') or {}).get('value')
print(f"{sys.argv[2]} flags={sys.argv[3]} value={d['value']:.2f}" + (f" train={t:.3f}" if t else ''))
PY
done
