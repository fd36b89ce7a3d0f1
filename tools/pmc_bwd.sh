#!/bin/bash
# PMC passes over the MSDA backward kernels at the config-4 encoder call
# (tools/msda_bwd_probe.py --case encoder: the direct-atomic kernel and the automatic choice),
# one rocprofv3 run per counter group under a hard kill; summaries gpurun_out/pmc_bwd<TAG>_<i>.json
export TMPDIR=/tmp
tag=${PMC_TAG:-}
i=0
for g in "SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_BUSY_CYCLES" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM SQ_INSTS_SALU" "FETCH_SIZE" "WRITE_SIZE"; do
  d=gpurun_out/pmc_bwd_raw_$i
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $g --output-format csv -d $d -o run -- python tools/msda_bwd_probe.py --iters 2 --case encoder > $d.log 2>&1 || exit 2
  python tools/pmc_summary.py gpurun_out/pmc_bwd${tag}_$i.json $d && rm -rf $d
  i=$((i+1))
done
