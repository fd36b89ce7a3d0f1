# Memory-pipeline PMC passes over the config-2 encoder sampler (tools/bench_msda.py --hm --rec
# --order --batch 16): texture addresser / data, L1 (TCP) and L2 (TCC) activity, one rocprofv3
# run per group (block limits: 2 TA, 2 TD, 4 TCP, 4 TCC, 2 GRBM)
export TMPDIR=/tmp
mkdir -p gpurun_out
i=0
for g in "TA_BUSY_avr TA_TA_BUSY_sum GRBM_GUI_ACTIVE" "TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE" "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum" "TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum GRBM_GUI_ACTIVE"; do
  d=gpurun_out/pmc_m_$i
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $g --output-format csv -d "$d" -o run -- python tools/bench_msda.py --iters 5 --hm --rec --order --batch 16 > "$d.log" 2>&1 || { echo "group $i failed"; tail -5 $d.log; exit 1; }
  python tools/pmc_summary.py gpurun_out/pmc_m_$i.json "$d" && rm -rf "$d"
  i=$((i+1))
done
