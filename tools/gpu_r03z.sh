# final round-3 check on HEAD: GPU suite, smoke, bench line
mkdir -p gpurun_out && export TMPDIR=/tmp && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03z_gputest.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03z_smoke.log 2>&1 && \
timeout -k 10 600 python bench.py > gpurun_out/r03z_bench.log 2>&1 && grep '^{' gpurun_out/r03z_bench.log > gpurun_out/r03z_bench.json
