#!/bin/bash
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u - > gpurun_out/r04ab_diag.log 2>&1 <<'PY'
import sys, traceback
sys.path.insert(0, 'tests')
import torch
import test_autograd_gpu as T
fails = 0
for i in range(20):
    try:
        T.test_conv_fwd_bwd(128, 512, 1, 1, 0, True, True, True, False)
    except AssertionError as e:
        fails += 1
        print('iter', i, 'FAIL', str(e).split('\n')[0], flush=True)
print('fails', fails, 'of 20', flush=True)
PY
echo "diag rc=$?"
tail -25 gpurun_out/r04ab_diag.log
timeout -k 10 300 python -u -m pytest tests/test_autograd_gpu.py -q --timeout 120 --timeout-method thread > gpurun_out/r04ab_autograd.log 2>&1; echo "autograd rc=$?"; tail -5 gpurun_out/r04ab_autograd.log
