#!/bin/bash
# round-4 v: direct 3x3 conv 128 -> 128: tests, kernel timing, bench A/B
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gemm_gpu.py -k "conv3x3 or big_conv" > gpurun_out/r04v_tests.log 2>&1 || { echo "tests failed rc=$?"; tail -30 gpurun_out/r04v_tests.log; exit 1; }
tail -2 gpurun_out/r04v_tests.log
timeout -k 10 120 python -u - > gpurun_out/r04v_time.log 2>&1 <<'PY' || { echo "timing failed"; tail gpurun_out/r04v_time.log; exit 1; }
import torch
from kinet_amd import kernels as K, _native
x = torch.relu(torch.randn(16, 100, 167, 128, device='cuda')).bfloat16()
w = K.pack_conv_weight(torch.randn(128, 128, 3, 3, device='cuda') * 0.03, torch.bfloat16)
sc, bi = torch.ones(128, device='cuda'), torch.zeros(128, device='cuda')
def t(flag, n=30):
    old = _native.lib().kinet_gemm_set_flags(flag)
    K.conv2d_nhwc(x, w, 1, 1, scale=sc, bias=bi, relu=True)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        K.conv2d_nhwc(x, w, 1, 1, scale=sc, bias=bi, relu=True)
    e.record(); torch.cuda.synchronize()
    _native.lib().kinet_gemm_set_flags(old)
    return s.elapsed_time(e) / n * 1e3
fl = 2 * 16 * 100 * 167 * 128 * 1152
for r in range(3):
    a, b = t(0), t(4096)
    print(f'stage-2 conv2 3x3 128->128 batch 16: direct {a:.1f} us ({fl / a / 1e6:.0f} TF/s) | implicit GEMM {b:.1f} us ({fl / b / 1e6:.0f} TF/s)')
PY
cat gpurun_out/r04v_time.log
bench() {  # tag args...
  local tag=$1; shift
  timeout -k 10 200 python -u bench.py --no-train --no-cpu-baseline --no-config5 --steps 30 "$@" > gpurun_out/r04v_$tag.log 2>&1 || { echo "bench $tag rc=$?"; tail -5 gpurun_out/r04v_$tag.log; exit 1; }
  python -c "import json; d=json.loads([l for l in open('gpurun_out/r04v_$tag.log') if l.startswith('{')][0]); f=d['device_ms_per_step_by_family']; s=d['roofline_gemm_conv_split']; print('$tag', round(d['value'],1), 'frames/s | conv', f.get('conv'), 'kxk', round(s['conv_kxk']['frac'],3))"
}
for i in 1 2; do
  bench c128_$i
  bench gemm_$i --gemm-flags 4096
done
