"""Build the kinet_amd native library in-tree: every kinet_amd/csrc/*.hip is compiled
for gfx950 with hipcc and linked into kinet_amd/_lib/libkinet_amd.so (a plain C-ABI
shared object: include/*.h).  The .so travels to the GPU box with the repo snapshot.

    python -m kinet_amd.build [--force] [-j N]
"""
import argparse
import concurrent.futures as cf
import glob
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, 'csrc')
OUT_DIR = os.path.join(HERE, '_lib')
OBJ_DIR = os.path.join(OUT_DIR, 'obj')
LIB = os.path.join(OUT_DIR, 'libkinet_amd.so')
HIPCC = os.environ.get('HIPCC', '/opt/rocm/bin/hipcc')
ARCH = 'gfx950'
FLAGS = ['--offload-arch=' + ARCH, '-O3', '-std=c++17', '-fPIC', '-Wall', '-Wno-unused-function',
         '-Wno-unused-variable', '-Wno-unused-but-set-variable']


def _sources():
    return sorted(glob.glob(os.path.join(CSRC, '*.hip')))


def _headers():
    return glob.glob(os.path.join(CSRC, '*.h')) + glob.glob(os.path.join(HERE, '..', 'include', '*.h'))


def _compile(src, force):
    obj = os.path.join(OBJ_DIR, os.path.basename(src) + '.o')
    newest_dep = max([os.path.getmtime(src)] + [os.path.getmtime(h) for h in _headers()])
    if not force and os.path.exists(obj) and os.path.getmtime(obj) >= newest_dep:
        return obj, False
    cmd = [HIPCC] + FLAGS + ['-c', src, '-o', obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f'hipcc failed for {src}:\n{r.stdout}\n{r.stderr}')
    return obj, True


def build(force=False, jobs=None, verbose=True):
    os.makedirs(OBJ_DIR, exist_ok=True)
    srcs = _sources()
    jobs = jobs or min(8, len(srcs)) or 1
    with cf.ThreadPoolExecutor(jobs) as ex:
        results = list(ex.map(lambda s: _compile(s, force), srcs))
    objs = [o for o, _ in results]
    rebuilt = any(r for _, r in results)
    if rebuilt or force or not os.path.exists(LIB):
        cmd = [HIPCC, '--offload-arch=' + ARCH, '-shared', '-fPIC', '-o', LIB] + objs
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f'link failed:\n{r.stdout}\n{r.stderr}')
        if verbose:
            print(f'[kinet_amd] built {LIB} from {len(srcs)} sources')
    return LIB


if __name__ == '__main__':
    ap = argparse.ArgumentParser()
    ap.add_argument('--force', action='store_true')
    ap.add_argument('-j', type=int, default=None)
    a = ap.parse_args()
    build(a.force, a.j)
    sys.exit(0)
