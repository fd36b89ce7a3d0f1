#!/bin/bash
# round-4 i: bottleneck-pair tests + A/B (D=64 LDS-resident kernel)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gemm_gpu.py -k "bottleneck" > gpurun_out/r04j_pair_tests.log 2>&1 || { echo "pair tests failed rc=$?"; tail -30 gpurun_out/r04j_pair_tests.log; exit 1; }
tail -3 gpurun_out/r04j_pair_tests.log
timeout -k 10 300 python -u tools/bneck_ab.py > gpurun_out/r04j_bneck_ab.log 2>&1 || { echo "ab failed"; tail -20 gpurun_out/r04j_bneck_ab.log; exit 1; }
cat gpurun_out/r04j_bneck_ab.log
