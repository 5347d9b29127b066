"""Build provenance: the source hash libRenderCore_MI355X.so carries in lh2_version() ("srchash=<16 hex>").

The Makefile (csrc/Makefile, HASH_SRCS / SRC_HASH) hashes the concatenated csrc/ and include/ sources in
make's $(sort) order, then the build flags; `source_hash()` recomputes the same digest from the checked-out files, and
`library_hash()` reads the one compiled into a library file without loading it (so a stale library can
be detected, and rebuilt, before any process maps it).
"""
from __future__ import annotations

import hashlib
import pathlib
import re

PKG = pathlib.Path(__file__).resolve().parent
CSRC = PKG / "csrc"
LIB_PATH = PKG / "libRenderCore_MI355X.so"


def _hash_sources() -> list[pathlib.Path]:
    names = []
    for pat in ("*.hip", "*.cpp", "*.h", "*.inc", "Makefile"):
        names += [p.name for p in CSRC.glob(pat)]
    for pat in ("*.h", "*.hpp"):
        names += ["../../include/" + p.name for p in (PKG.parent / "include").glob(pat)]
    # make's $(sort) is a byte-wise sort that also drops duplicates
    return [(CSRC / n) for n in sorted(set(names), key=lambda s: s.encode())]


def source_hash(extra: str = "", slp: str = "-fno-slp-vectorize", arch: str = "gfx950") -> str:
    """The hash of the sources and of the default build flags (csrc/Makefile EXTRA, SLP, ARCH)."""
    h = hashlib.sha256()
    for p in _hash_sources():
        h.update(p.read_bytes())
    h.update(f"flags:{extra}|{slp}|{arch}\n".encode())
    return h.hexdigest()[:16]


def library_hash(path: str | pathlib.Path = LIB_PATH) -> str | None:
    p = pathlib.Path(path)
    if not p.exists():
        return None
    m = re.search(rb"srchash=([0-9a-f]{16})", p.read_bytes())
    return m.group(1).decode() if m else None
