"""Build libftmi.so (the HIP C-ABI library) in-tree for gfx950.

    python -m forwardtacotron_amd.build        # incremental
    python -m forwardtacotron_amd.build --force

Each ``csrc/*.hip`` is compiled to an object with ``hipcc --offload-arch=gfx950`` and the
objects are linked into ``forwardtacotron_amd/libftmi.so``.  The library exports only the
``extern "C"`` entry points declared in ``include/ftmi.h``.  It cross-compiles without a GPU.
"""
from __future__ import annotations

import argparse
import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent
CSRC = PKG / 'csrc'
OBJ = PKG / 'build_obj'
LIB = PKG / 'libftmi.so'
ARCH = os.environ.get('FTMI_ARCH', 'gfx950')
HIPCC = os.environ.get('HIPCC', shutil.which('hipcc') or '/opt/rocm/bin/hipcc')
CFLAGS = ['-O3', '-std=c++17', '-fPIC', f'--offload-arch={ARCH}', '-Wall',
          '-Wno-unused-function', '-Wno-unused-variable', '-I', str(ROOT / 'include')]


def _sources():
    return sorted(CSRC.glob('*.hip'))


def _deps():
    return sorted(list(CSRC.glob('*.h')) + [ROOT / 'include' / 'ftmi.h'])


def _stale(target: Path, deps) -> bool:
    if not target.exists():
        return True
    t = target.stat().st_mtime
    return any(d.stat().st_mtime > t for d in deps)


def _compile(src: Path, force: bool, extra) -> Path:
    obj = OBJ / (src.stem + '.o')
    if force or _stale(obj, [src] + _deps()):
        cmd = [HIPCC, *CFLAGS, *extra, '-c', str(src), '-o', str(obj)]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f'hipcc failed for {src.name}:\n{r.stdout}\n{r.stderr}')
        if r.stderr.strip():
            sys.stderr.write(r.stderr)
    return obj


def build(force: bool = False, verbose: bool = False, extra=()) -> Path:
    """Compile every HIP source for gfx950 and link libftmi.so; returns the library path."""
    OBJ.mkdir(exist_ok=True)
    srcs = _sources()
    with ThreadPoolExecutor(max_workers=min(8, len(srcs))) as ex:
        objs = list(ex.map(lambda s: _compile(s, force, list(extra)), srcs))
    if force or _stale(LIB, objs):
        tmp = LIB.with_suffix('.so.tmp')
        cmd = [HIPCC, '-shared', f'--offload-arch={ARCH}', '-fPIC', *map(str, objs), '-o', str(tmp)]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f'link failed:\n{r.stdout}\n{r.stderr}')
        os.replace(tmp, LIB)
        if verbose:
            print(f'built {LIB}')
    return LIB


def build_stamps() -> Path:
    """Diagnostic library libftmi_stamps.so: the recurrence kernel with s_memtime phase
    stamps (-DFTMI_RNN_STAMPS).  Never loaded by the package unless FTMI_LIB points at it."""
    out = PKG / 'libftmi_stamps.so'
    objs = []
    for src in _sources():
        obj = OBJ / (src.stem + ('_stamps.o' if src.stem == 'rnn' else '.o'))
        if src.stem == 'rnn':
            cmd = [HIPCC, *CFLAGS, '-DFTMI_RNN_STAMPS', '-c', str(src), '-o', str(obj)]
            r = subprocess.run(cmd, capture_output=True, text=True)
            if r.returncode != 0:
                raise RuntimeError(r.stderr)
        else:
            _compile(src, False, [])
        objs.append(obj)
    r = subprocess.run([HIPCC, '-shared', f'--offload-arch={ARCH}', '-fPIC', *map(str, objs), '-o',
                        str(out)], capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(r.stderr)
    return out


if __name__ == '__main__':
    ap = argparse.ArgumentParser()
    ap.add_argument('--force', action='store_true')
    ap.add_argument('--stamps', action='store_true', help='also build libftmi_stamps.so')
    a = ap.parse_args()
    print(build(force=a.force, verbose=True))
    if a.stamps:
        print(build_stamps())
