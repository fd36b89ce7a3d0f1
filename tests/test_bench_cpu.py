"""bench.py's multi-rank launch path on the CPU: `--gpus 2` without an external launcher
starts two ranks itself (gloo stand-in for RCCL) and reports n_gpus = 2; under
torch.distributed.run the rank count comes from the launcher and must equal --gpus."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(cmd, env=None):
    e = dict(os.environ, **(env or {}))
    e.pop('WORLD_SIZE', None)
    r = subprocess.run(cmd, cwd=REPO, env=e, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith('{')]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


def test_bench_gpus2_spawns_two_ranks():
    line = _run([sys.executable, 'bench.py', '--cpu-stub', '--gpus', '2', '--steps', '3', '--warmup', '1',
                 '--batch', '4'])
    assert line['n_gpus'] == 2 and line['world_size'] == 2


def test_bench_under_torchrun():
    line = _run([sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node', '2',
                 '--master-addr', '127.0.0.1', '--master-port', '29517', 'bench.py', '--cpu-stub', '--gpus', '2',
                 '--steps', '2', '--warmup', '1', '--batch', '4'])
    assert line['n_gpus'] == 2


def test_bench_gpus1_single_process():
    line = _run([sys.executable, 'bench.py', '--cpu-stub', '--steps', '2', '--warmup', '1', '--batch', '4'])
    assert line['n_gpus'] == 1
