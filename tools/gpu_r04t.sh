#!/bin/bash
# round-4 t: max-pool + layer1[0] conv1 / downsample in one launch: tests, bench A/B
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gemm_gpu.py -k "pool_conv1x1 or backbone or stem" > gpurun_out/r04t_tests.log 2>&1 || { echo "tests failed rc=$?"; tail -30 gpurun_out/r04t_tests.log; exit 1; }
tail -2 gpurun_out/r04t_tests.log
bench() {  # tag args...
  local tag=$1; shift
  timeout -k 10 200 python -u bench.py --no-train --no-cpu-baseline --no-config5 --steps 30 "$@" > gpurun_out/r04t_$tag.log 2>&1 || { echo "bench $tag rc=$?"; tail -5 gpurun_out/r04t_$tag.log; exit 1; }
  python -c "import json; d=json.loads([l for l in open('gpurun_out/r04t_$tag.log') if l.startswith('{')][0]); f=d['device_ms_per_step_by_family']; print('$tag', round(d['value'],1), 'frames/s | conv', f.get('conv'), 'maxpool', f.get('kinet_maxpool2d_3x3s2'))"
}
for i in 1 2; do
  bench pp1_$i --pool-pair 1
  bench pp0_$i --pool-pair 0
done
