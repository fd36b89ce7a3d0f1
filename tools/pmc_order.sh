export TMPDIR=/tmp
for o in "" "--order"; do
  timeout -k 10 60 python tools/bench_msda.py $o 2>&1 | grep msda
  for c in FETCH_SIZE "TCC_HIT_sum TCC_MISS_sum"; do
    d=gpurun_out/pmo; rm -rf $d
    timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $d -o run -- python tools/bench_msda.py --iters 5 $o > /dev/null 2>&1 || exit 99
    python tools/pmc_summary.py gpurun_out/pmo_$o.json $d > /dev/null && python -c "
import json; d=json.load(open('gpurun_out/pmo_$o.json'))
for k,v in d['counters'].items():
    if 'msda' in k: print('$o', {a:(round(b/v['dispatches']) if isinstance(b,float) else b) for a,b in v.items()})"
  done
done
