#!/bin/bash
# round-4 m: pair tests (incl. the stage-1 -> stage-2 pair) + kernel A/B + bench A/B (A B A B)
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gemm_gpu.py -k "bottleneck" > gpurun_out/r04m_pair_tests.log 2>&1 || { echo "pair tests failed rc=$?"; tail -30 gpurun_out/r04m_pair_tests.log; exit 1; }
tail -2 gpurun_out/r04m_pair_tests.log
timeout -k 10 300 python -u tools/bneck_ab.py --reps 2 > gpurun_out/r04m_bneck_ab.log 2>&1 || { echo "ab failed"; tail -20 gpurun_out/r04m_bneck_ab.log; exit 1; }
cat gpurun_out/r04m_bneck_ab.log
for i in 1 2; do
  for p in 1 0; do
    timeout -k 10 200 python -u bench.py --no-train --no-cpu-baseline --no-config5 --steps 30 --bneck-pairs $p > gpurun_out/r04m_ab_p${p}_$i.log 2>&1 || { echo "bench rc=$?"; tail -5 gpurun_out/r04m_ab_p${p}_$i.log; exit 1; }
    python -c "import json,sys; d=json.loads([l for l in open('gpurun_out/r04m_ab_p${p}_$i.log') if l.startswith('{')][0]); print('pairs=$p run $i', round(d['value'],1), 'frames/s', d['device_ms_per_step_by_family'])"
  done
done
