# round-6 A/B batch: bottleneck pair widths, frame-shared pos, config-5 encoder strips (short bench runs,
# interleaved A B A B on one box), then the default bench line
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
step() { local name=$1 secs=$2; shift 2; timeout -k 10 "$secs" "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -o '"value": *[0-9.]*' gpurun_out/$name.log | head -1; if [ $rc -ne 0 ]; then tail -5 gpurun_out/$name.log; exit $rc; fi; }
q="--no-train --no-config3 --no-config5 --no-cpu-baseline --steps 20 --warmup 5"
for r in 1 2; do
  step r06c_pw64_$r 240 python -u bench.py $q --pair-widths 64 --detail gpurun_out/r06c_pw64_$r.json
  step r06c_pwall_$r 240 python -u bench.py $q --pair-widths 64,128,256 --detail gpurun_out/r06c_pwall_$r.json
  step r06c_pw256_$r 240 python -u bench.py $q --pair-widths 64,256 --detail gpurun_out/r06c_pw256_$r.json
  step r06c_pos0_$r 240 python -u bench.py $q --pair-widths 64 --share-pos 0 --detail gpurun_out/r06c_pos0_$r.json
done
c5="--workload config5 --no-train --no-cpu-baseline --steps 8 --warmup 2"
for r in 1 2; do
  step r06c_c5s0_$r 300 python -u bench.py $c5 --detail gpurun_out/r06c_c5s0_$r.json
  step r06c_c5s16_$r 300 python -u bench.py $c5 --enc-strips 16 --detail gpurun_out/r06c_c5s16_$r.json
  step r06c_c5s32_$r 300 python -u bench.py $c5 --enc-strips 32 --detail gpurun_out/r06c_c5s32_$r.json
done
step r06c_track_hz 300 python -u tools/track_hz.py
step r06c_kinet_track_hz 300 python -u tools/kinet_track_hz.py
