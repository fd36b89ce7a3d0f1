# round-6 evidence on the final defaults: smoke, then the profile round (kernel stats, PMC traffic, MFMA PMC, bench line)
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06f_smoke.log 2>&1 || { echo smoke failed; tail -5 gpurun_out/r06f_smoke.log; exit 98; }
tail -2 gpurun_out/r06f_smoke.log
bash tools/profile_round.sh r06f 10
