#!/bin/bash
# PMC passes over the head-major encoder kernel (tools/bench_msda.py --hm), one rocprofv3 run
# per counter group, each under a hard kill; summaries in gpurun_out/pmc_enc<TAG>_<i>.json
export TMPDIR=/tmp
groups=(
  "SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_BUSY_CYCLES"
  "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM SQ_INSTS_SALU"
  "TA_BUSY_avr TA_TA_BUSY_sum"
  "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum"
  "TD_BUSY_sum TD_TC_STALL_sum"
  "TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum"
  "FETCH_SIZE"
)
tag=${PMC_TAG:-}
i=0
for g in "${groups[@]}"; do
  d=gpurun_out/pmc_enc_raw_$i
  rm -rf "$d"
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $g --output-format csv -d "$d" -o run -- python tools/bench_msda.py --iters 5 "$@" > "$d.log" 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "[pmc_enc] group $i rc=$rc"; tail -3 "$d.log"; case $rc in 134|139) exit 99;; esac; fi
  python tools/pmc_summary.py gpurun_out/pmc_enc${tag}_$i.json "$d" && rm -rf "$d"
  i=$((i+1))
done
