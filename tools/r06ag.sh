# round-6: fragments read further ahead -- bottleneck pair (2048 = PF 1, 4096 = PF 2) and fused FFN (4 = PF 1)
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/pair_pf_probe.py --reps 3 > gpurun_out/r06ag_pair.log 2>&1 || { cat gpurun_out/r06ag_pair.log; exit 9; }
grep -v amdgpu gpurun_out/r06ag_pair.log
