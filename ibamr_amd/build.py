"""Build recipe for libibtk_le.so (gfx950) -- plain hipcc, in-tree.

The library is a C-ABI shared object (include/ibtk_le.h) with no torch
dependency; Python reaches it through ctypes (ibamr_amd/_lib.py).  Objects are
rebuilt only when a source or header is newer than the object.

Flags: -ffp-contract=off keeps every multiply and add separately rounded, as in
the Fortran (and the oracle), so parity can be bitwise.
"""
from __future__ import annotations

import os
import subprocess
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent
CSRC = PKG / "csrc"
# IBTK_LE_VARIANT=<name> with IBTK_LE_DEFS="-DNAME=V ..." builds an experiment
# into lib/var/<name>/ (load it with IBTK_LE_LIB); the default build ignores both.
_VAR = os.environ.get("IBTK_LE_VARIANT", "")
_LIBDIR = PKG / "lib" / "var" / _VAR if _VAR else PKG / "lib"
OBJ = _LIBDIR / "obj"
LIB = _LIBDIR / "libibtk_le.so"
INCLUDE = ROOT / "include"

SOURCES = ["le_hot.hip", "le_sweep.hip", "le_aux.hip", "le_bdry.hip", "le_sort.hip", "le_abi.cpp", "le_fortran.cpp", "le_interactor.cpp"]
ARCH = os.environ.get("IBTK_LE_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
CFLAGS = ["-O3", "-fPIC", "-std=c++17", "-ffp-contract=off", f"--offload-arch={ARCH}", f"-I{INCLUDE}",
          f"-I{CSRC}", "-Wall", "-Wno-unused-function", "-Wno-unused-variable", "-Wno-unused-value", "-Wno-unused-result"]
if _VAR:
    CFLAGS += os.environ.get("IBTK_LE_DEFS", "").split()


def _headers():
    return list(CSRC.glob("*.h")) + list(INCLUDE.rglob("*.h"))


def _stale(obj: Path, src: Path) -> bool:
    if not obj.exists():
        return True
    t = obj.stat().st_mtime
    return any(p.stat().st_mtime > t for p in [src, *_headers(), Path(__file__)])


def source_hash() -> str:
    """sha256 (16 hex digits) of the sources and headers the library is built from:
    ties a recorded profile (profiles/pmc_*.json) to the build it measured."""
    import hashlib
    h = hashlib.sha256()
    for f in sorted([*(CSRC / n for n in SOURCES), *_headers()], key=lambda q: str(q.relative_to(ROOT))):
        if f.exists():
            h.update(str(f.relative_to(ROOT)).encode())
            h.update(f.read_bytes())
    return h.hexdigest()[:16]


def build(verbose: bool = False) -> Path:
    OBJ.mkdir(parents=True, exist_ok=True)
    procs = []
    objs = []
    for name in SOURCES:
        src = CSRC / name
        if not src.exists():
            continue
        obj = OBJ / (name + ".o")
        objs.append(obj)
        if _stale(obj, src):
            lang = ["-x", "hip"] if name.endswith(".hip") else []
            cmd = [HIPCC, *CFLAGS, *lang, "-c", str(src), "-o", str(obj)]
            if verbose:
                print(" ".join(cmd), flush=True)
            procs.append((name, subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)))
    failed = []
    for name, p in procs:
        out, _ = p.communicate()
        if p.returncode != 0:
            failed.append((name, out.decode(errors="replace")))
        elif verbose and out:
            print(out.decode(errors="replace"))
    if failed:
        msg = "\n".join(f"--- {n} ---\n{o}" for n, o in failed)
        raise RuntimeError(f"hipcc failed:\n{msg}")
    if not LIB.exists() or any(o.stat().st_mtime > LIB.stat().st_mtime for o in objs):
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(LIB), *map(str, objs)]
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
        if r.returncode != 0:
            raise RuntimeError("link failed:\n" + r.stdout.decode(errors="replace"))
    return LIB


if __name__ == "__main__":
    print(build(verbose="-v" in sys.argv))
