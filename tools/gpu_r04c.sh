# round-4 gate of the records MSDA path + direct 3x3 conv: their tests first, the A/B timings,
# then the whole GPU suite, smoke and the default bench line
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/rec_debug.py > gpurun_out/r04c_rec_debug.log 2>&1; rc=$?; head -50 gpurun_out/r04c_rec_debug.log; case $rc in 0|1) ;; *) exit 90;; esac
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -k "records or direct_conv or tile_variants" > gpurun_out/r04c_new.log 2>&1; rc=$?; tail -12 gpurun_out/r04c_new.log; case $rc in 0|1) ;; *) exit 99;; esac
timeout -k 10 200 python -u tools/rec_ab.py > gpurun_out/r04c_rec_ab.log 2>&1 || exit 97
cat gpurun_out/r04c_rec_ab.log
timeout -k 10 200 python -u tools/conv_ab.py --iters 20 > gpurun_out/r04c_conv_ab.log 2>&1 || exit 98
head -12 gpurun_out/r04c_conv_ab.log
timeout -k 10 120 python -u tools/ffn_probe.py --rows 355568 --iters 10 > gpurun_out/r04c_ffn_probe.log 2>&1 || exit 96
cat gpurun_out/r04c_ffn_probe.log
# bench A/B (no train / config5 / cpu legs): default, 8x32-row FFN tile, 8-wave GEMM tiles everywhere
for v in "base:" "ffn4:--ffn-knob 4" "g2:--gemm-flags 2"; do
  n=${v%%:*}; args=${v#*:}
  timeout -k 10 240 python -u bench.py --steps 20 --warmup 5 --no-train --no-config5 --no-cpu-baseline $args > gpurun_out/r04c_ab_$n.log 2>&1 || exit 95
  grep -o '"value": [0-9.]*' gpurun_out/r04c_ab_$n.log | head -1 | sed "s/^/[$n] /"
done
