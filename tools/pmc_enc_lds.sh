export TMPDIR=/tmp
mkdir -p gpurun_out
i=0
for g in "SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_BUSY_CYCLES" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_SMEM" "SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_SCA SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_BRANCH SQ_INSTS_VALU_CVT SQ_WAVES GRBM_GUI_ACTIVE"; do
  d=gpurun_out/pmc_e_$i
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $g --output-format csv -d "$d" -o run -- python tools/bench_msda.py --iters 5 --hm --rec --order --batch 16 > "$d.log" 2>&1 || { echo "group $i failed"; tail -5 $d.log; exit 1; }
  python tools/pmc_summary.py gpurun_out/pmc_e_$i.json "$d" && rm -rf "$d"
  i=$((i+1))
done
