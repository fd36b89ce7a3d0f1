# round-3 evidence on HEAD (run from the repo root under gpurun): GPU suite, smoke, config-2
# profile + PMC + bench line (tools/profile_round.sh), config-5 bench line
mkdir -p gpurun_out && export TMPDIR=/tmp && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03u_gputest.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03u_smoke.log 2>&1 && \
bash tools/profile_round.sh r03u 10 && \
timeout -k 10 400 python bench.py --workload config5 --steps 10 --warmup 3 --no-cpu-baseline --no-train > gpurun_out/r03u_config5.log 2>&1 && \
grep '^{' gpurun_out/r03u_config5.log > gpurun_out/r03u_config5_bench.json
