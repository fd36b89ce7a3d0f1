# round-6: where the fused FFN's time goes (config-2 encoder FFN at batch 28): timing-only knobs
# (1 = no weight DMA after the prologue, 65 = also no per-chunk barrier; results garbage) + SQ PMC passes
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/ffn_probe.py --rows 622244 --iters 10 --knobs 0,1,65,0 > gpurun_out/r06ae_ffn.log 2>&1 || { cat gpurun_out/r06ae_ffn.log; exit 9; }
grep -v amdgpu gpurun_out/r06ae_ffn.log
bash tools/pmc_probe.sh ffn tools/ffn_probe.py --rows 622244 --iters 3 --knobs 0 || exit 9
python - <<'PY'
import json
for i in (0, 1):
    d = json.load(open(f'gpurun_out/pmc_ffn_{i}.json'))
    for k, v in d['counters'].items():
        if 'ffn' in k:
            print(i, k[:60], {c: round(x) for c, x in v.items()})
    for k, v in d['kernels'].items():
        if 'ffn' in k:
            print(i, k[:60], v)
PY
