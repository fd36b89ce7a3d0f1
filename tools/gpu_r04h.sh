#!/bin/bash
# round-4 h: bottleneck-pair tests + A/B, then the encoder PMC passes
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gemm_gpu.py -k "bottleneck" > gpurun_out/r04h_pair_tests.log 2>&1 || { echo "pair tests failed rc=$?"; tail -30 gpurun_out/r04h_pair_tests.log; exit 1; }
tail -3 gpurun_out/r04h_pair_tests.log
timeout -k 10 300 python -u tools/bneck_ab.py > gpurun_out/r04h_bneck_ab.log 2>&1 || { echo "ab failed"; tail -20 gpurun_out/r04h_bneck_ab.log; exit 1; }
cat gpurun_out/r04h_bneck_ab.log
PMC_TAG=_r04h timeout -k 10 400 bash tools/pmc_enc.sh --rec --batch 16 --order
