#!/bin/bash
# PMC passes (one rocprofv3 run per counter group) over tools/bench_msda.py; summaries in
# gpurun_out/pmc_msda<PMC_TAG>_<i>.json (PMC_GROUPS="0 2" restricts the groups).
# usage: tools/pmc_msda.sh [bench_msda args]
export TMPDIR=/tmp
groups=(
  "SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_LDS SQ_BUSY_CYCLES"
  "TA_BUSY_avr"
  "TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum"
  "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum"
  "TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum"
  "FETCH_SIZE"
)
tag=${PMC_TAG:-}
i=0
for g in "${groups[@]}"; do
  if [ -n "${PMC_GROUPS:-}" ] && [[ " $PMC_GROUPS " != *" $i "* ]]; then i=$((i+1)); continue; fi
  d=gpurun_out/pmc_msda_raw_$i
  rm -rf "$d"
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $g --output-format csv -d "$d" -o run -- python tools/bench_msda.py --iters 5 "$@" > "$d.log" 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "[pmc_msda] group $i rc=$rc"; tail -5 "$d.log"; case $rc in 124|137|134|139) exit 99;; esac; fi
  python tools/pmc_summary.py gpurun_out/pmc_msda${tag}_$i.json "$d" && rm -rf "$d"
  i=$((i+1))
done
