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


def test_compact_line_fits_driver_tail():
    """bench.py's stdout line (compact_line) keeps the driver contract's keys and every roofline /
    sub-benchmark number while staying well under the driver's ~8.7 KB stdout tail: built from the
    full record of round 5's HEAD run (profiles/r05end_bench.json, the largest line so far)."""
    import importlib.util
    here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location('bench_mod', os.path.join(here, 'bench.py'))
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    full = json.load(open(os.path.join(here, 'profiles', 'r05end_bench.json')))
    line = b.compact_line(full, 'gpurun_out/bench_detail.json')
    text = json.dumps(line, separators=(',', ':'))
    assert len(text) < 7000, len(text)
    for k in ('metric', 'value', 'unit', 'n_gpus', 'steps', 'warmup', 'ms_per_step', 'higher_is_better', 'scaling',
              'vs_baseline', 'dtype', 'data', 'config', 'roofline', 'cpu_baseline'):
        assert k in line, k
    r = line['roofline']
    assert r['bound'] == 'hbm' and 0 < r['frac'] < 1 and r['peak'] == 8000.0
    assert {'ms', 'prep_ms', 'sampler_ms', 'frac'} <= set(r['encoder_call'])
    assert line['roofline_mfma']['pmc_mfma_busy']['ffn_fused'] > 0
    assert line['config3']['value'] > 0 and line['config5']['msda_roofline']['frac'] > 0
    assert line['train']['value'] > 0 and line['cpu_baseline']['cores'] >= 1
