for d in 0 2 4; do KINET_ENC_DBG=$d timeout -k 10 60 python tools/bench_msda.py --batch 16 --order --hm --iters 30 2>&1 | grep -v amdgpu | sed "s/^/dbg=$d /" || exit 99; done
for n in 1 2 4; do timeout -k 10 60 python tools/bench_msda.py --batch 16 --order --hm --iters 30 --noise $n 2>&1 | grep -v amdgpu || exit 99; done
