#!/bin/bash
# Generic SQ/LDS PMC passes (one rocprofv3 run per counter group, nothing else beside --pmc)
# over a short python program; per-kernel summaries in gpurun_out/pmc_<tag>_<i>.json.
# usage: tools/pmc_probe.sh TAG script.py [args]
export TMPDIR=/tmp
tag=$1; shift
groups=(
  "SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_BUSY_CYCLES"
  "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_MFMA GRBM_GUI_ACTIVE GRBM_COUNT"
)
i=0
for g in "${groups[@]}"; do
  d=gpurun_out/pmc_${tag}_raw_$i
  rm -rf "$d"
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $g --output-format csv -d "$d" -o run -- python "$@" > "$d.log" 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "[pmc_probe] group $i rc=$rc"; tail -5 "$d.log"; exit 99; fi
  python tools/pmc_summary.py gpurun_out/pmc_${tag}_$i.json "$d" && rm -rf "$d"
  i=$((i+1))
done
