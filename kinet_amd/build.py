"""Build the kinet_amd native library in-tree: every kinet_amd/csrc/*.hip is compiled
for gfx950 with hipcc and linked into kinet_amd/_lib/libkinet_amd.so (a plain C-ABI
shared object: include/*.h).  The .so travels to the GPU box with the repo snapshot.

    python -m kinet_amd.build [--force] [-j N]
"""
import argparse
import concurrent.futures as cf
import glob
import hashlib
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


def source_hash():
    """sha256 over every kernel source and header (csrc/*.hip, csrc/*.h, include/*.h), by
    relative path and content.  Embedded in the library (kinet_version()) so a test on the
    GPU box can prove the .so it loaded was built from the sources it shipped with."""
    files = sorted(_sources() + _headers(), key=lambda p: os.path.relpath(p, os.path.dirname(HERE)))
    h = hashlib.sha256()
    for p in files:
        h.update(os.path.relpath(os.path.realpath(p), os.path.dirname(HERE)).encode() + b'\0')
        with open(p, 'rb') as f:
            h.update(f.read())
        h.update(b'\0')
    return h.hexdigest()[:16]


def _includes(path, seen=None):
    """The quoted #include files of `path`, transitively (the headers a TU can depend on)."""
    import re
    seen = set() if seen is None else seen
    with open(path) as f:
        for ln in f:
            m = re.match(r'\s*#\s*include\s+"([^"]+)"', ln)
            if m:
                q = os.path.normpath(os.path.join(os.path.dirname(path), m.group(1)))
                if q not in seen and os.path.exists(q):
                    seen.add(q)
                    _includes(q, seen)
    return seen


def _file_key(src):
    """Hash of one translation unit's inputs: its source + the headers it includes + the flags."""
    h = hashlib.sha256(' '.join(FLAGS).encode())
    for p in [src] + sorted(_includes(src)):
        with open(p, 'rb') as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def _compile(src, force, src_hash):
    """Content-addressed: an object is rebuilt unless its stamp matches the hash of its
    inputs (mtimes are not trusted -- a snapshot copy or checkout can reorder them).
    status.hip carries the whole-library hash, so it is keyed on that."""
    obj = os.path.join(OBJ_DIR, os.path.basename(src) + '.o')
    stamp = obj + '.hash'
    key = src_hash if os.path.basename(src) == 'status.hip' else _file_key(src)
    if not force and os.path.exists(obj) and os.path.exists(stamp) and open(stamp).read().strip() == key:
        return obj, False
    cmd = [HIPCC] + FLAGS + [f'-DKINET_SRC_HASH="{src_hash}"', '-c', src, '-o', obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f'hipcc failed for {src}:\n{r.stdout}\n{r.stderr}')
    with open(stamp, 'w') as f:
        f.write(key + '\n')
    return obj, True


def build(force=False, jobs=None, verbose=True):
    os.makedirs(OBJ_DIR, exist_ok=True)
    srcs = _sources()
    jobs = jobs or min(8, len(srcs)) or 1
    src_hash = source_hash()
    with cf.ThreadPoolExecutor(jobs) as ex:
        results = list(ex.map(lambda s: _compile(s, force, src_hash), srcs))
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
