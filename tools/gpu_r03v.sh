# PMC counter groups over the strip encoder kernel (config-2 encoder call, batch 16)
mkdir -p gpurun_out && export TMPDIR=/tmp && \
timeout -k 10 120 python tools/bench_msda.py --hm --order --batch 16 --iters 20 > gpurun_out/r03v_enc_time.log 2>&1 && \
PMC_TAG=_r03v bash tools/pmc_enc.sh --hm --order --batch 16 > gpurun_out/r03v_pmc_enc.log 2>&1
