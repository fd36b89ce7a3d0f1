#!/bin/bash
# Round evidence on the GPU box (run from the repo root under gpurun):
#   1. rocprofv3 --kernel-trace --stats of the default bench command (config 2 headline +
#      config-5 sub-run + config-4 train leg) -> gpurun_out/<tag>_kernel_stats.csv
#   2. per workload (config2, config3, config5) two PMC passes (FETCH_SIZE, WRITE_SIZE; separate runs,
#      --pmc with --kernel-trace only: no sys / runtime / hip / hsa / memory-copy trace domains)
#      of that workload ALONE (--no-train --no-config5 --no-config3)
#      -> gpurun_out/<tag>_<wl>_pmc_{fetch,write}.json -> per-launch HBM bytes merged into
#      gpurun_out/pmc_traffic.json under '<wl>:<kernel>' (also copied to profiles/ of this
#      snapshot so step 3 reads it)
#   3. the full bench line (incl. cpu_baseline) -> gpurun_out/<tag>_bench.json
# Every GPU step has its own time limit; a crash/timeout ends the script.
# usage: tools/profile_round.sh TAG [bench steps]
set -u
tag=$1; steps=${2:-10}
export TMPDIR=/tmp
run() { local secs=$1; shift; timeout -k 10 "$secs" "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "[profile_round] rc=$rc: $*"; exit 99; fi; }
rm -rf gpurun_out/prof_$tag
run 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$tag -o run -- python bench.py --steps "$steps" --warmup 3 --no-cpu-baseline > gpurun_out/${tag}_prof.log 2>&1
cp gpurun_out/prof_$tag/run_kernel_stats.csv gpurun_out/${tag}_kernel_stats.csv
python tools/pmc_summary.py gpurun_out/${tag}_trace_summary.json gpurun_out/prof_$tag
# all vs isolated (single-stream) dispatches: the cross-check of the bench line's HIP-event roofline
python tools/trace_isolated.py gpurun_out/prof_$tag gpurun_out/${tag}_trace_isolated.json > gpurun_out/${tag}_trace_isolated.txt 2>&1
rm -rf gpurun_out/prof_$tag
tf=gpurun_out/pmc_traffic.json
rm -f $tf
for wl in config2 config3 config5; do
  rm -rf gpurun_out/pmcf_$tag gpurun_out/pmcw_$tag
  one=(python bench.py --workload $wl --steps 2 --warmup 1 --no-cpu-baseline --no-train --no-config5 --no-config3)
  run 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcf_$tag -o run -- "${one[@]}" > gpurun_out/${tag}_${wl}_pmcf.log 2>&1
  run 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmcw_$tag -o run -- "${one[@]}" > gpurun_out/${tag}_${wl}_pmcw.log 2>&1
  python tools/pmc_summary.py gpurun_out/${tag}_${wl}_pmc_fetch.json gpurun_out/pmcf_$tag
  python tools/pmc_summary.py gpurun_out/${tag}_${wl}_pmc_write.json gpurun_out/pmcw_$tag
  rm -rf gpurun_out/pmcf_$tag gpurun_out/pmcw_$tag
  python tools/pmc_traffic.py gpurun_out/${tag}_${wl}_pmc_fetch.json gpurun_out/${tag}_${wl}_pmc_write.json $tf \
    "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE passes of '${one[*]}', round tag $tag" $wl
done
cp $tf profiles/pmc_traffic.json
# MFMA-pipe utilisation of the config-2 forward's kernels (one SQ + one GRBM counter: one pass)
rm -rf gpurun_out/pmcm_$tag
one=(python bench.py --workload config2 --steps 2 --warmup 1 --no-cpu-baseline --no-train --no-config5 --no-config3)
run 300 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmcm_$tag -o run -- "${one[@]}" > gpurun_out/${tag}_config2_pmcm.log 2>&1
python tools/pmc_summary.py gpurun_out/${tag}_config2_pmc_mfma_raw.json gpurun_out/pmcm_$tag
rm -rf gpurun_out/pmcm_$tag
python tools/pmc_mfma.py gpurun_out/pmc_mfma.json gpurun_out/${tag}_config2_pmc_mfma_raw.json \
  "rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE of '${one[*]}', round tag $tag"
cp gpurun_out/pmc_mfma.json profiles/pmc_mfma.json
run 600 python bench.py --steps "$steps" --warmup 3 > gpurun_out/${tag}_bench.log 2>&1
grep '^{' gpurun_out/${tag}_bench.log > gpurun_out/${tag}_bench.json
echo "[profile_round] done $tag"
