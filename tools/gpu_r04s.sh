#!/bin/bash
# round-4 s: fused stem + max-pool: tests, bench A/B, then the full gate (GPU suite, smoke, bench)
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gemm_gpu.py -k "stem" > gpurun_out/r04s_tests.log 2>&1 || { echo "tests failed rc=$?"; tail -30 gpurun_out/r04s_tests.log; exit 1; }
tail -2 gpurun_out/r04s_tests.log
bench() {  # tag args...
  local tag=$1; shift
  timeout -k 10 200 python -u bench.py --no-train --no-cpu-baseline --no-config5 --steps 30 "$@" > gpurun_out/r04s_$tag.log 2>&1 || { echo "bench $tag rc=$?"; tail -5 gpurun_out/r04s_$tag.log; exit 1; }
  python -c "import json; d=json.loads([l for l in open('gpurun_out/r04s_$tag.log') if l.startswith('{')][0]); f=d['device_ms_per_step_by_family']; print('$tag', round(d['value'],1), 'frames/s | conv', f.get('conv'), 'maxpool', f.get('kinet_maxpool2d_3x3s2'))"
}
for i in 1 2; do
  bench pool1_$i --stem-pool 1
  bench pool0_$i --stem-pool 0
done
bash tools/gpu_suite.sh r04s_gate
