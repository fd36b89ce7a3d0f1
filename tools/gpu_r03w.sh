# fused-FFN tile A/B inside the config-2 bench (3 streams): knob 0 (8 waves x 16 rows) vs 2 (4 waves x 32 rows)
mkdir -p gpurun_out && export TMPDIR=/tmp && : > gpurun_out/r03w_ffn_ab.txt && \
for k in 0 2 0 2; do
  timeout -k 10 240 python bench.py --steps 15 --warmup 3 --no-train --no-cpu-baseline --ffn-knob $k > gpurun_out/r03w_k$k.log 2>&1 || exit 99
  python -c "import json,sys; d=json.loads([l for l in open('gpurun_out/r03w_k$k.log') if l.startswith('{')][-1]); print('knob $k', round(d['value'],1), 'frames/s', round(d['ms_per_step'],3), 'ms/step')" >> gpurun_out/r03w_ffn_ab.txt
done
