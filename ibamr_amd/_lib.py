"""ctypes binding of libibtk_le.so (the C-ABI in include/ibtk_le.h).

The library is the product: there is no CPU fallback.  If it is missing or a
call fails, this module raises.
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path

_PKG = Path(__file__).resolve().parent
LIB_PATH = Path(os.environ.get("IBTK_LE_LIB", _PKG / "lib" / "libibtk_le.so"))

c_int = ctypes.c_int
c_double = ctypes.c_double
c_void_p = ctypes.c_void_p
P_int = ctypes.POINTER(ctypes.c_int)
P_double = ctypes.POINTER(ctypes.c_double)

STATUS = {
    0: "OK", 1: "UNKNOWN_KERNEL", 2: "GHOST_WIDTH", 3: "DEPTH", 4: "ARG", 5: "DEVICE", 6: "NOMEM", 7: "RANGE",
    8: "INVARIANT",
}

CENTERING = {"cell": 0, "side": 1, "node": 2, "edge": 3}


class IBTKLEError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"ibtk_le error {code} ({STATUS.get(code, '?')}): {msg}")
        self.code = code


class PatchGeom(ctypes.Structure):
    _fields_ = [
        ("ndim", c_int),
        ("ilower", c_int * 3),
        ("iupper", c_int * 3),
        ("gcw", c_int * 3),
        ("dx", c_double * 3),
        ("x_lower", c_double * 3),
        ("x_upper", c_double * 3),
        ("pitch", c_int * 2),
    ]

    @classmethod
    def make(cls, ilower, iupper, gcw, dx, x_lower, x_upper=None, pitch=None):
        nd = len(ilower)
        g = cls()
        g.ndim = nd
        if x_upper is None:
            x_upper = [x_lower[d] + (iupper[d] - ilower[d] + 1) * dx[d] for d in range(nd)]
        if isinstance(gcw, int):
            gcw = [gcw] * nd
        for d in range(nd):
            g.ilower[d] = int(ilower[d])
            g.iupper[d] = int(iupper[d])
            g.gcw[d] = int(gcw[d])
            g.dx[d] = float(dx[d])
            g.x_lower[d] = float(x_lower[d])
            g.x_upper[d] = float(x_upper[d])
        if pitch is not None:
            g.pitch[0], g.pitch[1] = int(pitch[0]), int(pitch[1])
        return g


_lib = None

# (name, restype, argtypes)
_SIGS = [
    ("ibtk_le_kernel_from_name", c_int, [ctypes.c_char_p]),
    ("ibtk_le_kernel_name", ctypes.c_char_p, [c_int]),
    ("ibtk_le_stencil_size", c_int, [c_int]),
    ("ibtk_le_min_ghost_width", c_int, [c_int]),
    ("ibtk_le_last_error", ctypes.c_char_p, []),
    ("ibtk_le_version", ctypes.c_char_p, []),
    ("ibtk_le_ctx_create", c_int, [c_int, c_void_p, ctypes.POINTER(c_void_p)]),
    ("ibtk_le_ctx_destroy", c_int, [c_void_p]),
    ("ibtk_le_ctx_set_stream", c_int, [c_void_p, c_void_p]),
    ("ibtk_le_ctx_synchronize", c_int, [c_void_p]),
    ("ibtk_le_ctx_enable_timing", c_int, [c_void_p, c_int]),
    ("ibtk_le_ctx_tune", c_int, [c_void_p, ctypes.c_char_p, c_int]),
    ("ibtk_le_ctx_set_plane_window", c_int, [c_void_p, c_int, c_int, c_int]),
    ("ibtk_le_ctx_last_kernel_ms", c_double, [c_void_p]),
    ("ibtk_le_ctx_count_adds", c_int, [c_void_p, c_int]),
    ("ibtk_le_wrap_positions", c_int, [c_void_p, c_int, ctypes.c_longlong, c_void_p, c_void_p, c_void_p, c_void_p]),
    ("ibtk_le_ctx_last_adds", c_int, [c_void_p, ctypes.POINTER(ctypes.c_ulonglong)]),
    ("ibtk_le_markers_create", c_int, [c_void_p, ctypes.POINTER(c_void_p)]),
    ("ibtk_le_markers_destroy", c_int, [c_void_p]),
    ("ibtk_le_markers_bin", c_int,
     [c_void_p, c_void_p, ctypes.POINTER(PatchGeom), c_int, c_void_p, c_void_p, c_void_p, c_int]),
    ("ibtk_le_markers_bin_count", c_int,
     [c_void_p, c_void_p, ctypes.POINTER(PatchGeom), c_int, c_void_p, c_int, c_void_p]),
    ("ibtk_le_markers_rebin", c_int, [c_void_p, c_void_p, c_void_p]),
    ("ibtk_le_markers_count", c_int, [c_void_p]),
    ("ibtk_le_markers_order", c_int, [c_void_p, ctypes.POINTER(c_void_p)]),
    ("ibtk_le_interp", c_int,
     [c_void_p, c_void_p, c_int, c_int, c_int, ctypes.POINTER(PatchGeom), ctypes.POINTER(c_void_p), c_int,
      c_void_p, c_int, c_void_p]),
    ("ibtk_le_spread", c_int,
     [c_void_p, c_void_p, c_int, c_int, c_int, ctypes.POINTER(PatchGeom), ctypes.POINTER(c_void_p), c_int,
      c_void_p, c_int, c_void_p]),
    ("ibtk_le_set_user_kernel", c_int, [c_void_p, c_int]),
    ("ibtk_le_user_kernel", c_int, [ctypes.POINTER(c_void_p), ctypes.POINTER(c_int)]),
    ("ibtk_le_user_interp", c_int,
     [c_void_p, c_int, c_int, ctypes.POINTER(PatchGeom), ctypes.POINTER(c_void_p), c_int, c_void_p, c_int, c_void_p,
      c_void_p, c_void_p, c_int]),
    ("ibtk_le_user_spread", c_int,
     [c_void_p, c_int, c_int, ctypes.POINTER(PatchGeom), ctypes.POINTER(c_void_p), c_int, c_void_p, c_int, c_void_p,
      c_void_p, c_void_p, c_int]),
    ("ibtk_le_spread_ds", c_int,
     [c_void_p, c_void_p, c_int, c_int, c_int, ctypes.POINTER(PatchGeom), ctypes.POINTER(c_void_p), c_int,
      c_void_p, c_int, c_void_p, c_void_p]),
    ("ibtk_le_fill_periodic_ghosts", c_int,
     [c_void_p, ctypes.POINTER(PatchGeom), c_int, ctypes.POINTER(c_void_p), c_int, c_void_p]),
    ("ibtk_le_fold_periodic_ghosts", c_int,
     [c_void_p, ctypes.POINTER(PatchGeom), c_int, ctypes.POINTER(c_void_p), c_int, c_void_p]),
    ("ibtk_le_local_numbering", c_int,
     [c_void_p, ctypes.POINTER(PatchGeom), c_void_p, c_int, c_void_p, ctypes.POINTER(c_int)]),
    ("ibtk_le_phys_bdry_side", c_int,
     [c_void_p, ctypes.POINTER(PatchGeom), ctypes.POINTER(c_void_p), c_void_p, c_void_p, c_void_p, c_void_p,
      c_int]),
    ("ibtk_le_position_update", c_int,
     [c_void_p, c_int, ctypes.c_longlong, c_double, c_void_p, c_void_p, c_void_p, c_void_p]),
    ("ibtk_le_slab_update_partition", c_int,
     [c_void_p, c_int, ctypes.c_longlong, c_double, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int,
      c_int, c_void_p, c_void_p]),
    ("ibtk_le_slab_update_partition_count", c_int,
     [c_void_p, c_int, ctypes.c_longlong, c_double, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int,
      c_int, c_void_p, c_void_p, c_void_p]),
    ("ibtk_le_slab_migrate_pack", c_int, [c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_int, c_void_p, c_void_p]),
    ("ibtk_le_slab_migrate_unpack", c_int,
     [c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_int, c_void_p]),
    ("ibtk_le_zero_ghosts", c_int, [c_void_p, ctypes.POINTER(PatchGeom), c_int, ctypes.POINTER(c_void_p), c_int]),
    ("ibtk_le_fill_interp", c_int,
     [c_void_p, c_void_p, c_int, c_int, c_int, ctypes.POINTER(PatchGeom), ctypes.POINTER(c_void_p), c_int, c_void_p,
      c_int, c_void_p, c_void_p]),
    ("ibtk_le_zero_ghosts_spread", c_int,
     [c_void_p, c_void_p, c_int, c_int, c_int, ctypes.POINTER(PatchGeom), ctypes.POINTER(c_void_p), c_int, c_void_p,
      c_int, c_void_p]),
    ("ibtk_le_zero_spread", c_int,
     [c_void_p, c_void_p, c_int, c_int, c_int, ctypes.POINTER(PatchGeom), ctypes.POINTER(c_void_p), c_int, c_void_p,
      c_int, c_void_p]),
    ("ibtk_le_mark_stencils", c_int,
     [c_void_p, c_void_p, c_int, c_int, c_int, ctypes.POINTER(PatchGeom), ctypes.POINTER(c_void_p), c_int,
      c_void_p]),
    ("ibtk_le_level_bin", c_int,
     [c_void_p, c_void_p, c_int, ctypes.POINTER(PatchGeom), c_int, c_void_p, ctypes.POINTER(c_int), c_void_p,
      c_void_p]),
    ("ibtk_le_level_interp", c_int,
     [c_void_p, c_void_p, c_int, c_int, c_int, ctypes.POINTER(c_void_p), c_int, c_void_p, c_int, c_void_p]),
    ("ibtk_le_level_spread", c_int,
     [c_void_p, c_void_p, c_int, c_int, c_int, ctypes.POINTER(c_void_p), c_int, c_void_p, c_int, c_void_p]),
    ("ibtk_le_level_zero_spread", c_int,
     [c_void_p, c_void_p, c_int, c_int, c_int, ctypes.POINTER(c_void_p), c_int, c_void_p, c_int, c_void_p]),
    ("ibtk_le_level_select_interior", c_int, [c_void_p, c_void_p, c_int, ctypes.POINTER(c_int), c_void_p]),
    ("ibtk_le_level_select_interior_reset", c_int, [c_void_p]),
    ("ibtk_le_level_fill_ghosts", c_int,
     [c_void_p, c_int, ctypes.POINTER(PatchGeom), c_int, ctypes.POINTER(c_void_p), c_int, c_void_p]),
    ("ibtk_le_level_fill_interp", c_int,
     [c_void_p, c_void_p, c_int, c_int, c_int, ctypes.POINTER(c_void_p), c_int, c_void_p, c_int, c_void_p, c_void_p]),
    ("ibtk_le_level_zero", c_int,
     [c_void_p, c_int, ctypes.POINTER(PatchGeom), c_int, ctypes.POINTER(c_void_p), c_int]),
    ("ibtk_le_index_set_list", c_int,
     [c_void_p, ctypes.POINTER(PatchGeom), c_void_p, c_void_p, c_int, c_int, c_void_p, c_int, c_void_p, c_void_p,
      c_int, ctypes.POINTER(c_int)]),
    ("ibtk_le_index_set_box_list", c_int,
     [c_void_p, ctypes.POINTER(PatchGeom), c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
      c_void_p, c_void_p, c_int, ctypes.POINTER(c_int)]),
    ("ibtk_le_list_in_box", c_int,
     [c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_int,
      ctypes.POINTER(c_int)]),
    ("ibtk_le_level_node_distribution", c_int,
     [c_void_p, c_int, ctypes.POINTER(PatchGeom), c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int,
      c_void_p, ctypes.POINTER(c_int), ctypes.POINTER(c_int)]),
    ("ibtk_le_level_index_lists", c_int,
     [c_void_p, c_int, ctypes.POINTER(PatchGeom), c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int,
      c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_int, c_void_p]),
    ("ibtk_le_ldata_reorder", c_int, [c_void_p, c_void_p, c_int, c_void_p, c_int, c_void_p]),
    ("ibtk_le_node_distribution", c_int,
     [c_void_p, ctypes.POINTER(PatchGeom), c_void_p, c_void_p, c_int, c_int, c_void_p, ctypes.POINTER(c_int),
      ctypes.POINTER(c_int)]),
    ("ibtk_le_periodic_index_list", c_int,
     [c_void_p, ctypes.POINTER(PatchGeom), c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p, c_int,
      ctypes.POINTER(c_int)]),
]

# Fortran-symbol shims and the C++ facade test hooks exported by the library.
FORTRAN_KERNELS = ["piecewise_constant", "discontinuous_linear", "piecewise_linear", "piecewise_cubic", "ib_3",
                   "ib_4", "ib_4_w8", "ib_6"]
FORTRAN_SYMBOLS = [f"lagrangian_{k}_{op}{d}d_" for k in FORTRAN_KERNELS for op in ("interp", "spread")
                   for d in (2, 3)]


def load():
    """Load the library (raises if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not LIB_PATH.exists():
        raise ImportError(f"libibtk_le.so not found at {LIB_PATH}; run __graft_entry__.build() "
                          f"or python -m ibamr_amd.build")
    lib = ctypes.CDLL(str(LIB_PATH))
    # an IBTK_LE_LIB override (an older build for an A/B run) may lack newer symbols
    lenient = "IBTK_LE_LIB" in os.environ
    for name, res, args in _SIGS:
        if lenient and not hasattr(lib, name):
            continue
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    _lib = lib
    return lib


def check(rc):
    if rc != 0:
        msg = load().ibtk_le_last_error().decode(errors="replace")
        raise IBTKLEError(rc, msg)
    return rc


def kernel_id(name: str) -> int:
    k = load().ibtk_le_kernel_from_name(name.encode())
    if k < 0:
        raise IBTKLEError(1, f"Unknown kernel function {name}")
    return k
