#!/bin/bash
# round-4 p: strided 1x1 downsample on the rw kernel + stem from the image: tests, A/B benches;
# MSDA backward phase breakdown; operating-point sweep
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gemm_gpu.py -k "strided_conv1x1 or stem or rw_conv or big_conv or bottleneck" > gpurun_out/r04p_tests.log 2>&1 || { echo "tests failed rc=$?"; tail -30 gpurun_out/r04p_tests.log; exit 1; }
tail -2 gpurun_out/r04p_tests.log
bench() {  # tag args...
  local tag=$1; shift
  timeout -k 10 200 python -u bench.py --no-train --no-cpu-baseline --no-config5 --steps 30 "$@" > gpurun_out/r04p_$tag.log 2>&1 || { echo "bench $tag rc=$?"; tail -5 gpurun_out/r04p_$tag.log; exit 1; }
  python -c "import json; d=json.loads([l for l in open('gpurun_out/r04p_$tag.log') if l.startswith('{')][0]); f=d['device_ms_per_step_by_family']; print('$tag', round(d['value'],1), 'frames/s | conv', f.get('conv'), 'pack', f.get('kinet_pack_image_kwfold'))"
}
for i in 1 2; do
  bench new_$i
  bench ds0_$i --gemm-flags 2048
  bench stem0_$i --stem-image 0
done
timeout -k 10 300 python -u tools/msda_bwd_probe.py --case encoder --phases > gpurun_out/r04p_bwd_phases.log 2>&1 || { echo "bwd probe failed"; tail -5 gpurun_out/r04p_bwd_phases.log; exit 1; }
cat gpurun_out/r04p_bwd_phases.log
for cfg in "24 3" "32 2" "16 4"; do
  set -- $cfg
  bench b$1_s$2 --batch $1 --streams $2
done
