#!/bin/bash
# round-4 q: MSDA backward list walk on 16-byte records; stem-from-image build v2: tests, probe, A/B, full line
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_msda_gpu.py tests/test_gemm_gpu.py -k "backward or stem" > gpurun_out/r04q_tests.log 2>&1 || { echo "tests failed rc=$?"; tail -30 gpurun_out/r04q_tests.log; exit 1; }
tail -2 gpurun_out/r04q_tests.log
timeout -k 10 300 python -u tools/msda_bwd_probe.py --phases > gpurun_out/r04q_bwd_phases.log 2>&1 || { echo "bwd probe failed"; tail -5 gpurun_out/r04q_bwd_phases.log; exit 1; }
cat gpurun_out/r04q_bwd_phases.log
bench() {  # tag args...
  local tag=$1; shift
  timeout -k 10 200 python -u bench.py --no-train --no-cpu-baseline --no-config5 --steps 30 "$@" > gpurun_out/r04q_$tag.log 2>&1 || { echo "bench $tag rc=$?"; tail -5 gpurun_out/r04q_$tag.log; exit 1; }
  python -c "import json; d=json.loads([l for l in open('gpurun_out/r04q_$tag.log') if l.startswith('{')][0]); f=d['device_ms_per_step_by_family']; print('$tag', round(d['value'],1), 'frames/s | conv', f.get('conv'), 'pack', f.get('kinet_pack_image_kwfold'))"
}
for i in 1 2; do
  bench stem1_$i --stem-image 1
  bench stem0_$i --stem-image 0
done
timeout -k 10 600 python -u bench.py > gpurun_out/r04q_full.log 2>&1 || { echo "full bench rc=$?"; tail -5 gpurun_out/r04q_full.log; exit 1; }
python -c "import json; d=json.loads([l for l in open('gpurun_out/r04q_full.log') if l.startswith('{')][0]); t=d['train']; print('full', round(d['value'],1), 'train', round(t['value'],2), 'bwd list ms', round(t['msda_bwd_roofline']['avg_launch_ms'],3), 'frac', round(t['msda_bwd_roofline']['frac'],4), 'config5', round(d['config5']['value'],1))"
