"""Identity of the HIP sources (no torch import): sha256 over csrc/*.hip, csrc/*.h and
include/ftmi.h.  build.py bakes it into libftmi.so (ftmi_build_id) and _lib.load refuses a
library whose id differs from the sources next to it, so a stale prebuilt binary can never
be loaded silently."""
from __future__ import annotations

import hashlib
from pathlib import Path

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent


def source_files():
    csrc = PKG / 'csrc'
    return sorted(list(csrc.glob('*.hip')) + list(csrc.glob('*.h'))) + [ROOT / 'include' / 'ftmi.h']


def source_hash() -> str:
    h = hashlib.sha256()
    for f in source_files():
        h.update(f.name.encode() + b'\0')
        h.update(f.read_bytes())
        h.update(b'\0')
    return h.hexdigest()
