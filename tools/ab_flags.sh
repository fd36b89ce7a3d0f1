# usage: bash tools/ab_flags.sh WORKLOAD FLAGS_A FLAGS_B [extra bench args]: A B A B bench runs
set -e
w=$1; fa=$2; fb=$3; shift 3
mkdir -p gpurun_out
for f in $fa $fb $fa $fb; do
  timeout -k 10 300 python -u bench.py --workload $w --no-cpu-baseline --gemm-flags $f "$@" > gpurun_out/ab_${w}_$f.log 2>&1
  echo "$w flags=$f $(grep -o '"value": [0-9.]*' gpurun_out/ab_${w}_$f.log | head -1)"
done
