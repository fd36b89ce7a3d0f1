#!/bin/bash
# SQ counters of the encoder-call MSDA kernels (old gather kernel vs LDS-window kernel).
export TMPDIR=/tmp
g="SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT"
for v in "--order" "--enc"; do
  d=gpurun_out/pmc_enc_raw${v//-/}
  rm -rf "$d"
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc $g --output-format csv -d "$d" -o run -- python tools/bench_msda.py --iters 5 --batch 8 $v > "$d.log" 2>&1 || { echo "rc=$? $v"; tail -5 "$d.log"; exit 99; }
  python tools/pmc_summary.py gpurun_out/pmc_enc${v//-/}.json "$d" && rm -rf "$d"
done
