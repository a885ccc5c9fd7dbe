"""Python host API over the C-ABI (device-resident torch tensors).

Thin, allocation-free wrappers: every array is a torch tensor on the GPU and is
handed to libibtk_le.so by pointer.  Arrays follow SAMRAI's Fortran layout, so a
3-D ghosted array of extents (n0, n1, n2) is a C-contiguous tensor of shape
(n2, n1, n0) [x fastest], with an extra leading depth axis for cell/node data.
"""
from __future__ import annotations

import ctypes
import math
import sys
from dataclasses import dataclass
from typing import Optional, Sequence

import numpy as np
import torch

from . import _lib
from ._lib import PatchGeom, check, kernel_id

CENTERING = _lib.CENTERING


def _ptr(t: Optional[torch.Tensor]):
    if t is None:
        return None
    if not t.is_cuda:
        raise ValueError("ibtk_le works on device-resident tensors")
    if not t.is_contiguous():
        raise ValueError("tensor must be contiguous")
    return ctypes.c_void_p(t.data_ptr())


def _ptr_array(ts: Sequence[torch.Tensor], geom: Optional["Geometry"] = None):
    """Pointer table of Eulerian arrays: contiguous, or laid out by ``geom``'s pitch."""
    arr = (ctypes.c_void_p * max(1, len(ts)))()
    for i, t in enumerate(ts):
        if t is None:
            arr[i] = None
            continue
        if t.dtype != torch.float64 or not t.is_cuda:
            raise ValueError("Eulerian arrays must be float64 device tensors")
        if geom is not None and geom.pitched:
            if not geom.has_layout(t):
                raise ValueError(f"array strides {t.stride()} do not follow the geometry's pitch {geom.pitch}")
        elif not t.is_contiguous():
            raise ValueError("Eulerian arrays must be contiguous (or follow the geometry's pitch)")
        arr[i] = t.data_ptr()
    return arr


@dataclass
class Geometry:
    """Patch box + ghost width + Cartesian geometry (one uniform patch)."""

    ilower: Sequence[int]
    iupper: Sequence[int]
    gcw: int | Sequence[int]
    dx: Sequence[float]
    x_lower: Sequence[float]
    x_upper: Optional[Sequence[float]] = None
    pitch: Optional[Sequence[int]] = None  # (row, plane) pitch of the arrays in elements; None = packed

    def __post_init__(self):
        self.ndim = len(self.ilower)
        if isinstance(self.gcw, int):
            self.gcw = [self.gcw] * self.ndim
        if self.x_upper is None:
            self.x_upper = [self.x_lower[d] + (self.iupper[d] - self.ilower[d] + 1) * self.dx[d]
                            for d in range(self.ndim)]
        if self.pitch is not None:
            self.pitch = (int(self.pitch[0]), int(self.pitch[1]))
        self.c = PatchGeom.make(self.ilower, self.iupper, self.gcw, self.dx, self.x_lower, self.x_upper,
                                self.pitch)

    @property
    def pitched(self) -> bool:
        return self.pitch is not None and tuple(self.pitch) != (0, 0)

    def aligned(self, align: int = 16) -> "Geometry":
        """The same patch with its arrays' rows padded to a multiple of `align` elements
        (ibtk_le_patch_geom::pitch): 128-byte rows for align 16 (3-D only)."""
        if self.ndim != 3:
            raise ValueError("a pitched layout needs a 3-D patch")
        n0 = self.iupper[0] - self.ilower[0] + 2 + 2 * self.gcw[0]
        n1 = self.iupper[1] - self.ilower[1] + 2 + 2 * self.gcw[1]
        return Geometry(self.ilower, self.iupper, self.gcw, self.dx, self.x_lower, self.x_upper,
                        ((n0 + align - 1) // align * align, n1))

    def strides(self, centering: str, comp: int = 0, depth: int = 1):
        """torch strides (elements) of component `comp`'s array."""
        shape = self.array_shape(centering, comp, depth)
        if not self.pitched:
            st, acc = [], 1
            for n in reversed(shape):
                st.append(acc)
                acc *= n
            return tuple(reversed(st))
        p0, p1 = self.pitch
        n = list(reversed(shape[-3:]))  # (n0, n1, n2)
        s2 = p0 * (p1 if p1 else n[1])
        st = (s2, p0, 1)
        return ((s2 * n[2],) + st) if len(shape) == 4 else st

    def has_layout(self, t: torch.Tensor) -> bool:
        """True if `t` is one of this geometry's arrays (shape and strides of some component)."""
        for cen in ("side", "cell", "node", "edge"):
            for c in range(self.ncomp(cen)):
                shape = self.array_shape(cen, c, t.shape[0] if t.dim() == 4 else 1)
                if tuple(t.shape) == tuple(shape) and tuple(t.stride()) == self.strides(cen, c, shape[0] if
                                                                                        len(shape) == 4 else 1):
                    return True
        return False

    @staticmethod
    def periodic_unit(N: Sequence[int], ghost: int, x_lower=None, x_upper=None):
        nd = len(N)
        xl = list(x_lower) if x_lower is not None else [0.0] * nd
        xu = list(x_upper) if x_upper is not None else [1.0] * nd
        dx = [(xu[d] - xl[d]) / N[d] for d in range(nd)]
        return Geometry([0] * nd, [n - 1 for n in N], ghost, dx, xl, xu)

    def array_shape(self, centering: str, comp: int = 0, depth: int = 1):
        """torch shape of the ghosted array of component `comp`."""
        ext = self.ext_mask(centering, comp)
        n = [self.iupper[d] - self.ilower[d] + 1 + 2 * self.gcw[d] + ((ext >> d) & 1) for d in range(self.ndim)]
        shape = tuple(reversed(n))
        return ((depth,) + shape) if centering in ("cell", "node") else shape

    def ext_mask(self, centering, comp=0):
        full = (1 << self.ndim) - 1
        return {"cell": 0, "node": full, "side": 1 << comp, "edge": full & ~(1 << comp)}[centering]

    def ncomp(self, centering):
        return self.ndim if centering in ("side", "edge") else 1

    def alloc(self, centering: str, depth: int = 1, device="cuda", fill=0.0):
        if not self.pitched:
            return [torch.full(self.array_shape(centering, c, depth), fill, dtype=torch.float64, device=device)
                    for c in range(self.ncomp(centering))]
        out = []
        for c in range(self.ncomp(centering)):
            shape = self.array_shape(centering, c, depth)
            st = self.strides(centering, c, depth)
            size = 1 + sum((n - 1) * s for n, s in zip(shape, st))
            buf = torch.full((size,), fill, dtype=torch.float64, device=device)  # allocator: 256-B aligned
            out.append(torch.as_strided(buf, shape, st))
        return out


class Context:
    """A library context bound to one device and a HIP stream (torch's current stream by default)."""

    def __init__(self, device: int = 0, stream: Optional[torch.cuda.Stream] = None):
        self.lib = _lib.load()
        self.device = device
        s = stream if stream is not None else torch.cuda.current_stream(device)
        self.stream = s
        h = ctypes.c_void_p()
        check(self.lib.ibtk_le_ctx_create(device, ctypes.c_void_p(s.cuda_stream), ctypes.byref(h)))
        self.h = h
        self.plane_window = (0, 0, -1)

    def set_stream(self, stream: torch.cuda.Stream):
        self.stream = stream
        check(self.lib.ibtk_le_ctx_set_stream(self.h, ctypes.c_void_p(stream.cuda_stream)))

    def synchronize(self):
        check(self.lib.ibtk_le_ctx_synchronize(self.h))

    def enable_timing(self, on=True):
        check(self.lib.ibtk_le_ctx_enable_timing(self.h, int(on)))

    def set_plane_window(self, mode: int, zlo: int = 0, zhi: int = -1):
        """Restrict the next 3-D sweeps to the items inside (1) / outside (2) the planes
        [zlo, zhi]; 0 = every item (ibtk_le_ctx_set_plane_window).  With mode 0 a
        window zlo <= zhi still cuts the sweep items of later binnings at its faces."""
        check(self.lib.ibtk_le_ctx_set_plane_window(self.h, int(mode), int(zlo), int(zhi)))
        self.plane_window = (int(mode), int(zlo), int(zhi))

    def tune(self, key: str, value: int):
        """Diagnostic overrides of the 3-D sweeps' work-item order (ibtk_le_ctx_tune)."""
        check(self.lib.ibtk_le_ctx_tune(self.h, key.encode(), int(value)))

    def last_kernel_ms(self) -> float:
        return float(self.lib.ibtk_le_ctx_last_kernel_ms(self.h))

    def count_adds(self, on=True):
        """Counted 3-D spread sweeps (ibtk_le_ctx_count_adds; syncs the host per launch)."""
        check(self.lib.ibtk_le_ctx_count_adds(self.h, int(on)))

    def last_adds(self):
        """(ds_add_f64 wave-instructions, lane adds) of the last counted spread call."""
        out = (ctypes.c_ulonglong * 2)()
        check(self.lib.ibtk_le_ctx_last_adds(self.h, out))
        return int(out[0]), int(out[1])

    def close(self):
        if getattr(self, "h", None):
            self.lib.ibtk_le_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        # at interpreter exit the HIP runtime may already be torn down: leave the
        # device memory to the process exit rather than free it into a dead runtime
        if sys.is_finalizing():
            return
        try:
            self.close()
        except Exception:
            pass


class Markers:
    """A binned marker list on the device (the device-side LIndexSetData)."""

    def __init__(self, ctx: Context):
        self.ctx = ctx
        h = ctypes.c_void_p()
        check(ctx.lib.ibtk_le_markers_create(ctx.h, ctypes.byref(h)))
        self.h = h
        self.kernel = None
        self.geom = None

    def bin(self, geom: Geometry, kernel: str, X: torch.Tensor, indices: Optional[torch.Tensor] = None,
            Xshift: Optional[torch.Tensor] = None, n: Optional[int] = None):
        if indices is not None:
            assert indices.dtype == torch.int32
            n = indices.numel()
        elif n is None:
            n = X.shape[0]
        if Xshift is not None:
            assert Xshift.dtype == torch.float64 and Xshift.numel() == n * geom.ndim
        assert X.dtype == torch.float64
        check(self.ctx.lib.ibtk_le_markers_bin(self.ctx.h, self.h, ctypes.byref(geom.c), kernel_id(kernel), _ptr(X),
                                               _ptr(indices), _ptr(Xshift), int(n)))
        self.kernel, self.geom, self.n = kernel, geom, n
        self._n_dev = None
        return self

    def bin_count(self, geom: Geometry, kernel: str, X: torch.Tensor, n_dev: torch.Tensor):
        """Bin the first n_dev[0] (a device int32) of X's rows (ibtk_le_markers_bin_count):
        a fixed-capacity marker array, no host sync."""
        if X.dtype != torch.float64 or not X.is_contiguous() or X.dim() != 2 or X.shape[1] != 3:
            raise ValueError("X: contiguous (capacity, 3) float64")
        if n_dev.dtype != torch.int32 or n_dev.numel() < 1 or not n_dev.is_cuda:
            raise ValueError("n_dev: a device int32")
        check(self.ctx.lib.ibtk_le_markers_bin_count(self.ctx.h, self.h, ctypes.byref(geom.c), kernel_id(kernel),
                                                     _ptr(X), int(X.shape[0]), _ptr(n_dev)))
        self.kernel, self.geom, self.n = kernel, geom, X.shape[0]
        # rebin() reads the count again on the device: keep its memory alive until the next bin
        self._n_dev = n_dev
        return self

    def rebin(self, X: torch.Tensor):
        """Re-bin the last binned list at new positions X (ibtk_le_markers_rebin): the
        same result as binning it again, computed from the previous order."""
        if self.kernel is None:
            raise RuntimeError("rebin: the list was never binned")
        assert X.dtype == torch.float64
        check(self.ctx.lib.ibtk_le_markers_rebin(self.ctx.h, self.h, _ptr(X)))
        return self

    def count(self) -> int:
        return int(self.ctx.lib.ibtk_le_markers_count(self.h))

    def order(self) -> torch.Tensor:
        """Canonical order (device int32 copy): order[i] = list position of the i-th sorted entry."""
        p = ctypes.c_void_p()
        check(self.ctx.lib.ibtk_le_markers_order(self.h, ctypes.byref(p)))
        n = self.count()
        out = torch.empty(n, dtype=torch.int32, device=f"cuda:{self.ctx.device}")
        if n:
            torch.cuda.current_stream(self.ctx.device).synchronize()
            self.ctx.synchronize()
            import ctypes as _c
            hip = _hip()
            check_hip(hip.hipMemcpy(_c.c_void_p(out.data_ptr()), p, _c.c_size_t(4 * n), 3))
        return out

    def close(self):
        if getattr(self, "h", None):
            self.ctx.lib.ibtk_le_markers_destroy(self.h)
            self.h = None

    def __del__(self):
        # at interpreter exit the HIP runtime may already be torn down: leave the
        # device memory to the process exit rather than free it into a dead runtime
        if sys.is_finalizing():
            return
        try:
            self.close()
        except Exception:
            pass


_hip_lib = None


def _hip():
    global _hip_lib
    if _hip_lib is None:
        _hip_lib = ctypes.CDLL("libamdhip64.so")
        _hip_lib.hipMemcpy.restype = ctypes.c_int
        _hip_lib.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    return _hip_lib


def check_hip(rc):
    if rc != 0:
        raise RuntimeError(f"hip error {rc}")


def interp(ctx: Context, markers: Markers, kernel: str, centering: str, geom: Geometry,
           q: Sequence[torch.Tensor], Q: torch.Tensor, X: torch.Tensor, q_depth: int = 1, Q_depth: Optional[int] = None,
           axis: int = 0):
    """Q(d, s) = sum w q  (LEInteractor::interpolate)."""
    if Q_depth is None:
        Q_depth = geom.ndim if centering in ("side", "edge") else q_depth
    arr = _ptr_array(q, geom)
    check(ctx.lib.ibtk_le_interp(ctx.h, markers.h, kernel_id(kernel), CENTERING[centering], axis,
                                 ctypes.byref(geom.c), arr, q_depth, _ptr(Q), Q_depth, _ptr(X)))


def spread(ctx: Context, markers: Markers, kernel: str, centering: str, geom: Geometry,
           q: Sequence[torch.Tensor], Q: torch.Tensor, X: torch.Tensor, q_depth: int = 1, Q_depth: Optional[int] = None,
           axis: int = 0, ds: Optional[torch.Tensor] = None):
    """q += S Q  (LEInteractor::spread), deterministic marker-ordered sums.

    With ``ds`` (one float64 per marker): q += S (Q ds), the density-weighted
    LDataManager::spread (LDataManager.cpp:398-470)."""
    if Q_depth is None:
        Q_depth = geom.ndim if centering in ("side", "edge") else q_depth
    arr = _ptr_array(q, geom)
    if ds is None:
        check(ctx.lib.ibtk_le_spread(ctx.h, markers.h, kernel_id(kernel), CENTERING[centering], axis,
                                     ctypes.byref(geom.c), arr, q_depth, _ptr(Q), Q_depth, _ptr(X)))
    else:
        if ds.dtype != torch.float64 or ds.numel() * Q_depth != Q.numel():
            raise ValueError("ds: one float64 per marker")
        check(ctx.lib.ibtk_le_spread_ds(ctx.h, markers.h, kernel_id(kernel), CENTERING[centering], axis,
                                        ctypes.byref(geom.c), arr, q_depth, _ptr(Q), Q_depth, _ptr(ds), _ptr(X)))


def fill_interp(ctx: Context, markers: Markers, kernel: str, centering: str, geom: Geometry,
                q: Sequence[torch.Tensor], Q: torch.Tensor, X: torch.Tensor, q_depth: int = 1,
                Q_depth: Optional[int] = None, axis: int = 0, periodic=None):
    """fill_periodic_ghosts(q, periodic) then interp, Q bit for bit, in one sweep on a 3-D
    column binning (ibtk_le_fill_interp): the ghost points are read at their periodic
    images and q is left unmodified."""
    if Q_depth is None:
        Q_depth = geom.ndim if centering in ("side", "edge") else q_depth
    arr = _ptr_array(q, geom)
    pa = _periodic_arg(periodic, geom.ndim)
    check(ctx.lib.ibtk_le_fill_interp(ctx.h, markers.h, kernel_id(kernel), CENTERING[centering], axis,
                                      ctypes.byref(geom.c), arr, q_depth, _ptr(Q), Q_depth, _ptr(X),
                                      pa[0] if pa else None))


def zero_ghosts_spread(ctx: Context, markers: Markers, kernel: str, centering: str, geom: Geometry,
                       q: Sequence[torch.Tensor], Q: torch.Tensor, X: torch.Tensor, q_depth: int = 1,
                       Q_depth: Optional[int] = None, axis: int = 0):
    """zero_ghosts(q) then spread, bit for bit, in one sweep on a 3-D column binning
    (ibtk_le_zero_ghosts_spread): the owned ghost points start from 0."""
    if Q_depth is None:
        Q_depth = geom.ndim if centering in ("side", "edge") else q_depth
    arr = _ptr_array(q, geom)
    check(ctx.lib.ibtk_le_zero_ghosts_spread(ctx.h, markers.h, kernel_id(kernel), CENTERING[centering], axis,
                                             ctypes.byref(geom.c), arr, q_depth, _ptr(Q), Q_depth, _ptr(X)))


def zero_spread(ctx: Context, markers: Markers, kernel: str, centering: str, geom: Geometry,
                q: Sequence[torch.Tensor], Q: torch.Tensor, X: torch.Tensor, q_depth: int = 1,
                Q_depth: Optional[int] = None, axis: int = 0):
    """q := 0 (every point, ghosts included) then spread, bit for bit: the target as
    LDataManager::spread hands it to LEInteractor::spread (LDataManager.cpp:596-660;
    ibtk_le_zero_spread).  On a 3-D column binning one sweep that writes q and never
    reads it."""
    if Q_depth is None:
        Q_depth = geom.ndim if centering in ("side", "edge") else q_depth
    arr = _ptr_array(q, geom)
    check(ctx.lib.ibtk_le_zero_spread(ctx.h, markers.h, kernel_id(kernel), CENTERING[centering], axis,
                                      ctypes.byref(geom.c), arr, q_depth, _ptr(Q), Q_depth, _ptr(X)))


# USER_DEFINED kernel function (LEInteractor::s_kernel_fcn, LEInteractor.h:100-101):
# a Python callable phi(r) -> float, called by the library on the host
USER_KERNEL_FN = ctypes.CFUNCTYPE(ctypes.c_double, ctypes.c_double)
_user_fn_ref = None  # the ctypes callback the library holds (kept alive here)


def set_user_kernel(fcn, stencil_size: int):
    """LEInteractor::s_kernel_fcn = fcn; s_kernel_fcn_stencil_size = stencil_size.
    fcn None restores the default (ib4_kernel_fcn, stencil 4)."""
    global _user_fn_ref
    lib = _lib.load()
    cb = USER_KERNEL_FN(fcn) if fcn is not None else None
    check(lib.ibtk_le_set_user_kernel(ctypes.cast(cb, ctypes.c_void_p) if cb is not None else None, int(stencil_size)))
    _user_fn_ref = cb


def _user_call(fn, ctx, centering, geom, q, Q, X, indices, xshift, q_depth, Q_depth, axis):
    if Q_depth is None:
        Q_depth = geom.ndim if centering in ("side", "edge") else q_depth
    n = indices.numel() if indices is not None else X.shape[0]
    if indices is not None and indices.dtype != torch.int32:
        raise ValueError("indices: int32")
    if xshift is not None and (xshift.dtype != torch.float64 or xshift.numel() != n * geom.ndim):
        raise ValueError("xshift: float64, NDIM per list entry")
    check(fn(ctx.h, CENTERING[centering], axis, ctypes.byref(geom.c), _ptr_array(q, geom), q_depth, _ptr(Q), Q_depth,
             _ptr(X), _ptr(indices), _ptr(xshift), n))


def user_interp(ctx: Context, centering: str, geom: Geometry, q: Sequence[torch.Tensor], Q: torch.Tensor,
                X: torch.Tensor, indices: Optional[torch.Tensor] = None, xshift: Optional[torch.Tensor] = None,
                q_depth: int = 1, Q_depth: Optional[int] = None, axis: int = 0):
    """Q(d, s) = sum w q with the USER_DEFINED kernel (LEInteractor::userDefinedInterpolate,
    LEInteractor.cpp:3141-3266) over the list (indices, xshift)."""
    _user_call(ctx.lib.ibtk_le_user_interp, ctx, centering, geom, q, Q, X, indices, xshift, q_depth, Q_depth, axis)


def user_spread(ctx: Context, centering: str, geom: Geometry, q: Sequence[torch.Tensor], Q: torch.Tensor,
                X: torch.Tensor, indices: Optional[torch.Tensor] = None, xshift: Optional[torch.Tensor] = None,
                q_depth: int = 1, Q_depth: Optional[int] = None, axis: int = 0):
    """q += S Q with the USER_DEFINED kernel (LEInteractor::userDefinedSpread,
    LEInteractor.cpp:3268-3393): every grid point summed in list order."""
    _user_call(ctx.lib.ibtk_le_user_spread, ctx, centering, geom, q, Q, X, indices, xshift, q_depth, Q_depth, axis)


class Level:
    """A level of 3-D patches binned together (ibtk_le_level_bin): LDataManager's
    patch loop (LDataManager.cpp:625-660, 763-807) as one launch per sweep.

    geoms: the patches' Geometry (one dx); lists[q]: patch q's list, either None
    (every marker) or (indices int32 device tensor, Xshift float64 device tensor
    or None).  interp/spread take the arrays of every patch, patch by patch
    (``arrays[q]`` = that patch's list of component arrays)."""

    def __init__(self, ctx: Context, geoms: Sequence[Geometry], kernel: str, X: torch.Tensor, lists):
        if len(geoms) != len(lists) or not geoms:
            raise ValueError("one list per patch")
        self.ctx, self.geoms, self.kernel = ctx, list(geoms), kernel
        self.markers = Markers(ctx)
        M = X.shape[0]
        idx, xs, off = [], [], [0]
        any_shift = any(l is not None and l[1] is not None for l in lists)
        for l in lists:
            if l is None:
                i = torch.arange(M, dtype=torch.int32, device=X.device)
                x = torch.zeros((M, 3), dtype=torch.float64, device=X.device)
            else:
                i = l[0].to(torch.int32)
                x = l[1] if l[1] is not None else torch.zeros((i.numel(), 3), dtype=torch.float64, device=X.device)
            idx.append(i)
            xs.append(x)
            off.append(off[-1] + i.numel())
        self.indices = torch.cat(idx).contiguous()
        self.xshift = torch.cat(xs).contiguous() if any_shift else None
        self._G = (PatchGeom * len(geoms))(*[g.c for g in geoms])
        self._O = (ctypes.c_int * len(off))(*off)
        self.bin(X)

    @classmethod
    def from_flat(cls, ctx: Context, geoms: Sequence[Geometry], kernel: str, X: torch.Tensor, indices: torch.Tensor,
                  xshift: Optional[torch.Tensor], offsets: Sequence[int]):
        """A level from the concatenated lists: patch q's entries are [offsets[q], offsets[q+1])."""
        self = cls.__new__(cls)
        self.ctx, self.geoms, self.kernel = ctx, list(geoms), kernel
        self.markers = Markers(ctx)
        self.indices = indices.to(torch.int32).contiguous()
        self.xshift = xshift.contiguous() if xshift is not None else None
        self._G = (PatchGeom * len(geoms))(*[g.c for g in geoms])
        self._O = (ctypes.c_int * len(offsets))(*[int(o) for o in offsets])
        self.bin(X)
        return self

    def relist(self, indices: torch.Tensor, xshift: Optional[torch.Tensor], offsets: Sequence[int]):
        """Replace the patches' lists (a regrid / redistribution; bin again after)."""
        if len(offsets) != len(self.geoms) + 1:
            raise ValueError("one offset per patch, plus the end")
        self.indices = indices.to(torch.int32).contiguous()
        self.xshift = xshift.contiguous() if xshift is not None else None
        self._O = (ctypes.c_int * len(offsets))(*[int(o) for o in offsets])
        return self

    def bin(self, X: torch.Tensor):
        """(Re-)bin the level's lists at positions X (ibtk_le_level_bin)."""
        check(self.ctx.lib.ibtk_le_level_bin(self.ctx.h, self.markers.h, len(self.geoms), self._G,
                                             kernel_id(self.kernel), _ptr(X), self._O, _ptr(self.indices),
                                             _ptr(self.xshift)))
        return self

    def rebin(self, X: torch.Tensor):
        """Re-bin the same lists at new positions X (ibtk_le_markers_rebin): the result
        of bin(X), computed from the previous order."""
        assert X.dtype == torch.float64
        check(self.ctx.lib.ibtk_le_markers_rebin(self.ctx.h, self.markers.h, _ptr(X)))
        return self

    def select_interior(self, n_markers: int, indices: torch.Tensor, offsets: Sequence[int],
                        lists_changed: bool = False):
        """After a bin on the ghost-box lists: later interps write Q only from the entries
        the interior lists (patch q: indices[offsets[q]:offsets[q+1]]) name
        (ibtk_le_level_select_interior); one binning serves both sweeps.

        The library keeps the selection while the same list (pointer, offsets, n_markers)
        comes back and no re-binning moved a marker.  A new tensor object drops it here; an
        int32 list rewritten IN PLACE and passed again is the same object, so say so with
        `lists_changed=True` (or call reset_selection() first)."""
        if len(offsets) != len(self.geoms) + 1:
            raise ValueError("one offset per patch, plus the end")
        idx = indices.to(torch.int32).contiguous()
        if lists_changed or idx is not getattr(self, "_sel", None):
            # another list object (possibly at the old list's address): the library's kept
            # selection is keyed on the pointer, so it is dropped here
            check(self.ctx.lib.ibtk_le_level_select_interior_reset(self.markers.h))
        self._sel = idx  # kept alive until the next bin
        O = (ctypes.c_int * len(offsets))(*[int(o) for o in offsets])
        check(self.ctx.lib.ibtk_le_level_select_interior(self.ctx.h, self.markers.h, int(n_markers), O, _ptr(idx)))
        return self

    def reset_selection(self):
        """Drop the kept interior selection (ibtk_le_level_select_interior_reset): the next
        select_interior recomputes it, e.g. after its interior list was edited in place."""
        check(self.ctx.lib.ibtk_le_level_select_interior_reset(self.markers.h))
        self._sel = None
        return self

    def fill_ghosts(self, centering: str, arrays, q_depth: int = 1, periodic=None):
        """Ghost fill across the level's patches (ibtk_le_level_fill_ghosts)."""
        pa = _periodic_arg(periodic, 3)
        check(self.ctx.lib.ibtk_le_level_fill_ghosts(self.ctx.h, len(self.geoms), self._G, CENTERING[centering],
                                                     self._arrays(arrays), q_depth, pa[0] if pa else None))

    def zero(self, centering: str, arrays, q_depth: int = 1):
        """Every patch array := 0, ghosts included, in one launch (ibtk_le_level_zero)."""
        check(self.ctx.lib.ibtk_le_level_zero(self.ctx.h, len(self.geoms), self._G, CENTERING[centering],
                                              self._arrays(arrays), q_depth))

    def _arrays(self, arrays):
        # the pointer table of a list of per-patch arrays, cached on the list object
        # (a level reuses its u and f arrays step after step); reused only when every
        # entry still has the device pointer it had, so an array replaced in place
        # (arrays[q] = new tensors) rebuilds the table
        key = id(arrays)
        flat = [t for per in arrays for t in per]
        ptrs = tuple(t.data_ptr() for t in flat)
        hit = self.__dict__.setdefault("_ptr_cache", {}).get(key)
        if hit is not None and hit[0] is arrays and hit[2] == ptrs:
            return hit[1]
        tab = _ptr_array(flat)
        self._ptr_cache[key] = (arrays, tab, ptrs)
        return tab

    def interp(self, centering: str, arrays, Q: torch.Tensor, X: torch.Tensor, q_depth: int = 1,
               Q_depth: Optional[int] = None, axis: int = 0):
        if Q_depth is None:
            Q_depth = 3 if centering in ("side", "edge") else q_depth
        check(self.ctx.lib.ibtk_le_level_interp(self.ctx.h, self.markers.h, kernel_id(self.kernel),
                                                CENTERING[centering], axis, self._arrays(arrays), q_depth, _ptr(Q),
                                                Q_depth, _ptr(X)))

    def fill_interp(self, centering: str, arrays, Q: torch.Tensor, X: torch.Tensor, q_depth: int = 1,
                    Q_depth: Optional[int] = None, axis: int = 0, periodic=None):
        """`fill_ghosts` then `interp`, Q bit for bit, in one sweep that reads each ghost point in
        the neighbour patch the fill would copy it from (ibtk_le_level_fill_interp); the two calls
        when a component's arrays do not lie within one 2-GB window (see `alloc_level`)."""
        if Q_depth is None:
            Q_depth = 3 if centering in ("side", "edge") else q_depth
        pa = _periodic_arg(periodic, 3)
        check(self.ctx.lib.ibtk_le_level_fill_interp(self.ctx.h, self.markers.h, kernel_id(self.kernel),
                                                     CENTERING[centering], axis, self._arrays(arrays), q_depth,
                                                     _ptr(Q), Q_depth, _ptr(X), pa[0] if pa else None))

    def spread(self, centering: str, arrays, Q: torch.Tensor, X: torch.Tensor, q_depth: int = 1,
               Q_depth: Optional[int] = None, axis: int = 0):
        if Q_depth is None:
            Q_depth = 3 if centering in ("side", "edge") else q_depth
        check(self.ctx.lib.ibtk_le_level_spread(self.ctx.h, self.markers.h, kernel_id(self.kernel),
                                                CENTERING[centering], axis, self._arrays(arrays), q_depth, _ptr(Q),
                                                Q_depth, _ptr(X)))

    def zero_spread(self, centering: str, arrays, Q: torch.Tensor, X: torch.Tensor, q_depth: int = 1,
                    Q_depth: Optional[int] = None, axis: int = 0):
        """`zero` then `spread` in one launch (ibtk_le_level_zero_spread): LDataManager::spread's
        setToScalar(f, 0, interior_only=false) fused with its patch loop; bitwise the two calls."""
        if Q_depth is None:
            Q_depth = 3 if centering in ("side", "edge") else q_depth
        check(self.ctx.lib.ibtk_le_level_zero_spread(self.ctx.h, self.markers.h, kernel_id(self.kernel),
                                                     CENTERING[centering], axis, self._arrays(arrays), q_depth,
                                                     _ptr(Q), Q_depth, _ptr(X)))


def alloc_level(geoms: Sequence[Geometry], centering: str, depth: int = 1, device="cuda"):
    """Per-patch arrays of a level (a list per patch, as Geometry.alloc gives), each component's
    arrays of every patch carved from one allocation: the layout ibtk_le_level_fill_interp reads
    across patches in one window."""
    per = [g.array_shape(centering, a, depth) for g in geoms for a in range(3 if centering in ("side", "edge") else 1)]
    ncomp = 3 if centering in ("side", "edge") else 1
    out = [[None] * ncomp for _ in geoms]
    for a in range(ncomp):
        sizes = [math.prod(per[q * ncomp + a]) for q in range(len(geoms))]
        # 16-byte aligned slices
        offs, tot = [], 0
        for n in sizes:
            offs.append(tot)
            tot += (n + 1) // 2 * 2
        block = torch.zeros(tot, dtype=torch.float64, device=device)
        for q in range(len(geoms)):
            out[q][a] = block[offs[q]:offs[q] + sizes[q]].view(per[q * ncomp + a])
    return out


def _periodic_arg(periodic, ndim):
    if periodic is None:
        return None
    a = (ctypes.c_int * 3)(*([int(bool(p)) for p in periodic] + [1] * (3 - ndim)))
    return ctypes.cast(a, ctypes.c_void_p), a


def fill_periodic_ghosts(ctx: Context, geom: Geometry, centering: str, q, q_depth=1, periodic=None):
    pa = _periodic_arg(periodic, geom.ndim)
    check(ctx.lib.ibtk_le_fill_periodic_ghosts(ctx.h, ctypes.byref(geom.c), CENTERING[centering], _ptr_array(q, geom),
                                               q_depth, pa[0] if pa else None))


def fold_periodic_ghosts(ctx: Context, geom: Geometry, centering: str, q, q_depth=1, periodic=None):
    pa = _periodic_arg(periodic, geom.ndim)
    check(ctx.lib.ibtk_le_fold_periodic_ghosts(ctx.h, ctypes.byref(geom.c), CENTERING[centering], _ptr_array(q, geom),
                                               q_depth, pa[0] if pa else None))


def zero_ghosts(ctx: Context, geom: Geometry, centering: str, q, q_depth=1):
    check(ctx.lib.ibtk_le_zero_ghosts(ctx.h, ctypes.byref(geom.c), CENTERING[centering], _ptr_array(q, geom), q_depth))


def local_numbering(ctx: Context, geom: Geometry, X: torch.Tensor):
    """LDataManager::computeNodeDistribution's local numbering for one patch, on the device.

    Returns (order, n_interior): order[i] = input index of the marker with local index i
    (cells of the patch box in box order, x fastest, input order within a cell; markers
    outside the box last, in input order)."""
    if X.dtype != torch.float64 or not X.is_cuda or not X.is_contiguous() or X.dim() != 2 or X.shape[1] != geom.ndim:
        raise ValueError("X: contiguous (M, ndim) float64 device tensor")
    n = X.shape[0]
    order = torch.empty(n, dtype=torch.int32, device=X.device)
    nin = ctypes.c_int(0)
    check(ctx.lib.ibtk_le_local_numbering(ctx.h, ctypes.byref(geom.c), _ptr(X), n, _ptr(order), ctypes.byref(nin)))
    return order, nin.value


def phys_bdry_side(ctx: Context, geom: Geometry, u, physical, acoef, bcoef, gcoef, adjoint: bool):
    """CartSideRobinPhysBdryOp on one patch of side data, on the device.

    adjoint=False: setPhysicalBoundaryConditions (CartSideRobinPhysBdryOp.cpp:358-422), the
    ghost fill before interp; adjoint=True: accumulateFromPhysicalBoundaryData (:429-493), the
    fold LDataManager::spread runs after spreading (LDataManager.cpp:655-659).
    physical[2 d + upper] flags a physical face; acoef/bcoef/gcoef broadcast to
    (ndim, 2 ndim) = [component axis, face location] (constant Robin coefficients per face)."""
    nd = geom.ndim
    if len(physical) != 2 * nd:
        raise ValueError("physical: one flag per face (2 ndim)")
    if len(u) != nd:
        raise ValueError("u: one side array per axis")
    g = geom.c.gcw[0]
    for a in range(nd):
        n = 1
        for d in range(nd):
            n *= geom.c.iupper[d] - geom.c.ilower[d] + 1 + 2 * g + (1 if d == a else 0)
        if u[a].numel() != n:
            raise ValueError(f"u[{a}]: {u[a].numel()} values, the ghosted side box holds {n}")
    phys = (ctypes.c_int * 6)(*([int(bool(p)) for p in physical] + [0] * (6 - 2 * nd)))
    coefs = []
    for c in (acoef, bcoef, gcoef):
        a = np.ascontiguousarray(np.broadcast_to(np.asarray(c, np.float64), (nd, 2 * nd)))
        coefs.append(a)
    cp = [a.ctypes.data_as(ctypes.c_void_p) for a in coefs]
    check(ctx.lib.ibtk_le_phys_bdry_side(ctx.h, ctypes.byref(geom.c), _ptr_array(u, geom), ctypes.cast(phys, ctypes.c_void_p),
                                         cp[0], cp[1], cp[2], int(bool(adjoint))))


UPDATE_SCHEMES = {"euler": 0, "midpoint": 1, "trapezoidal": 2}


def position_update(ctx: Context, scheme: str, dt: float, X: torch.Tensor, U0: torch.Tensor,
                    U1: Optional[torch.Tensor] = None, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """X_new = X + dt U0 ("euler", "midpoint") or (X + dt/2 U0) + dt/2 U1 ("trapezoidal"), on the device.

    IBMethod::eulerStep / midpointStep / trapezoidalStep (IBMethod.cpp:619-681).
    ``out`` may be ``X`` itself (in-place update).  Returns ``out``.
    """
    if scheme not in UPDATE_SCHEMES:
        raise ValueError(f"unknown scheme {scheme!r}")
    if scheme == "trapezoidal" and U1 is None:
        raise ValueError("trapezoidal needs U1")
    arrs = [X, U0] + ([U1] if scheme == "trapezoidal" else [])
    for t in arrs:
        if t.dtype != torch.float64 or t.shape != X.shape:
            raise ValueError("X, U0, U1 must be float64 of one shape")
    if out is None:
        out = torch.empty_like(X)
    elif out.shape != X.shape or out.dtype != torch.float64:
        raise ValueError("out must match X")
    check(ctx.lib.ibtk_le_position_update(ctx.h, UPDATE_SCHEMES[scheme], X.numel(), float(dt), _ptr(X), _ptr(U0),
                                          _ptr(U1) if scheme == "trapezoidal" else None, _ptr(out)))
    return out


def slab_update_partition(ctx: Context, scheme: str, dt: float, X: torch.Tensor, U0: torch.Tensor, L, Nz: int,
                          nranks: int, rank: int, U1: Optional[torch.Tensor] = None):
    """Position update fused with the z-slab migration classes (ibtk_le_slab_update_partition):
    (X_new wrapped into [0, L), order int32 [stay | to rank-1 | to rank+1 | further], counts
    int32 device tensor of 4)."""
    if scheme not in UPDATE_SCHEMES:
        raise ValueError(f"unknown scheme {scheme!r}")
    for t in [X, U0] + ([U1] if scheme == "trapezoidal" else []):
        if t is None or t.dtype != torch.float64 or t.shape != X.shape or X.dim() != 2 or X.shape[1] != 3:
            raise ValueError("X, U0, U1: (M, 3) float64 of one shape")
    M = X.shape[0]
    Xn = torch.empty_like(X)
    order = torch.empty(max(M, 1), dtype=torch.int32, device=X.device)
    counts = torch.zeros(4, dtype=torch.int32, device=X.device)
    Ld = (ctypes.c_double * 3)(*[float(v) for v in L])
    check(ctx.lib.ibtk_le_slab_update_partition(ctx.h, UPDATE_SCHEMES[scheme], M, float(dt), _ptr(X), _ptr(U0),
                                                _ptr(U1) if scheme == "trapezoidal" else None, _ptr(Xn),
                                                ctypes.cast(Ld, ctypes.c_void_p), int(Nz), int(nranks), int(rank),
                                                _ptr(order), _ptr(counts)))
    return Xn, order[:M], counts


def slab_update_partition_count(ctx: Context, scheme: str, dt: float, X: torch.Tensor, U0: torch.Tensor, L,
                                Nz: int, nranks: int, rank: int, n_dev: torch.Tensor,
                                U1: Optional[torch.Tensor] = None):
    """slab_update_partition over the first n_dev[0] rows of capacity-sized arrays
    (ibtk_le_slab_update_partition_count): (X_new, order, counts), all on the device."""
    if scheme not in UPDATE_SCHEMES:
        raise ValueError(f"unknown scheme {scheme!r}")
    for t in [X, U0] + ([U1] if scheme == "trapezoidal" else []):
        if t is None or t.dtype != torch.float64 or t.shape != X.shape or X.dim() != 2 or X.shape[1] != 3:
            raise ValueError("X, U0, U1: (capacity, 3) float64 of one shape")
    C = X.shape[0]
    Xn = torch.empty_like(X)
    order = torch.empty(max(C, 1), dtype=torch.int32, device=X.device)
    counts = torch.zeros(4, dtype=torch.int32, device=X.device)
    Ld = (ctypes.c_double * 3)(*[float(v) for v in L])
    check(ctx.lib.ibtk_le_slab_update_partition_count(ctx.h, UPDATE_SCHEMES[scheme], C, float(dt), _ptr(X), _ptr(U0),
                                                      _ptr(U1) if scheme == "trapezoidal" else None, _ptr(Xn),
                                                      ctypes.cast(Ld, ctypes.c_void_p), int(Nz), int(nranks),
                                                      int(rank), _ptr(n_dev), _ptr(order), _ptr(counts)))
    return Xn, order, counts


def slab_migrate_pack(ctx: Context, rows: torch.Tensor, order: torch.Tensor, counts: torch.Tensor,
                      send_down: torch.Tensor, send_up: torch.Tensor):
    """The down / up leavers of rows ([capacity, depth] float64) into the send buffers
    ([send_cap, depth] each), ibtk_le_slab_migrate_pack."""
    D = rows.shape[1]
    if send_down.shape != send_up.shape or send_down.shape[1] != D:
        raise ValueError("send buffers: (send_cap, depth) each")
    check(ctx.lib.ibtk_le_slab_migrate_pack(ctx.h, _ptr(rows), D, _ptr(order), _ptr(counts), send_down.shape[0],
                                            _ptr(send_down), _ptr(send_up)))


def slab_migrate_unpack(ctx: Context, rows: torch.Tensor, order: torch.Tensor, counts: torch.Tensor,
                        recv_counts: torch.Tensor, from_down: torch.Tensor, from_up: torch.Tensor,
                        out: torch.Tensor, n_out: torch.Tensor):
    """out = stayers, then the arrivals from below, then from above; n_out[0] = their
    number (ibtk_le_slab_migrate_unpack)."""
    D = rows.shape[1]
    if out.shape[1] != D or from_down.shape != from_up.shape:
        raise ValueError("buffer shapes")
    check(ctx.lib.ibtk_le_slab_migrate_unpack(ctx.h, _ptr(rows), D, _ptr(order), _ptr(counts), _ptr(recv_counts),
                                              _ptr(from_down), _ptr(from_up), from_down.shape[0], _ptr(out),
                                              out.shape[0], _ptr(n_out)))


def index_set_list(ctx: Context, geom: Geometry, X: torch.Tensor, ghost: int, lag: Optional[torch.Tensor] = None,
                   periodic=None, which: str = "all"):
    """LIndexSetData::cacheLocalIndices' lists on the device (ibtk_le_index_set_list):
    (indices int32, Xshift float64 [n, ndim]) in the reference's order (ghost-box
    cells in iteration order, Lagrangian index within a cell).  which: "all",
    "interior" or "ghost"."""
    M = X.shape[0]
    cnt = ctypes.c_int(0)
    pa = _periodic_arg(periodic, geom.ndim)
    w = {"all": 0, "interior": 1, "ghost": 2}[which]
    if lag is not None and (lag.dtype != torch.int32 or lag.numel() != M):
        raise ValueError("lag: one int32 per marker")
    cap = M * (3 ** geom.ndim) if ghost > 0 else M
    idx = torch.empty(max(1, cap), dtype=torch.int32, device=X.device)
    xs = torch.empty((max(1, cap), geom.ndim), dtype=torch.float64, device=X.device)
    check(ctx.lib.ibtk_le_index_set_list(ctx.h, ctypes.byref(geom.c), _ptr(X), _ptr(lag), M, ghost,
                                         pa[0] if pa else None, w, _ptr(idx), _ptr(xs), cap, ctypes.byref(cnt)))
    n = cnt.value
    return idx[:n].contiguous(), xs[:n].contiguous()


class _IntArg:
    """An int[3] argument kept alive with its c_void_p view."""

    def __init__(self, vals):
        self.a = (ctypes.c_int * 3)(*([int(v) for v in vals] + [0] * (3 - len(vals))))
        self.p = ctypes.cast(self.a, ctypes.c_void_p)


def _box_arg(lo, hi, ndim):
    if len(lo) != ndim or len(hi) != ndim:
        raise ValueError("box: ndim lower and upper cell indices")
    return _IntArg(lo), _IntArg(hi)


def index_set_box_list(ctx: Context, geom: Geometry, X: torch.Tensor, ghost: int, box_lo, box_hi,
                       lag: Optional[torch.Tensor] = None, periodic=None):
    """LEInteractor::buildLocalIndices for any box of cells (ibtk_le_index_set_box_list,
    LEInteractor.cpp:3070-3106): (indices int32, Xshift float64 [n, ndim], cells int32
    [n, ndim]), the entries of the all-nodes list whose cell lies in [box_lo, box_hi],
    in that list's order."""
    M = X.shape[0]
    cnt = ctypes.c_int(0)
    pa = _periodic_arg(periodic, geom.ndim)
    lo, hi = _box_arg(box_lo, box_hi, geom.ndim)
    if lag is not None and (lag.dtype != torch.int32 or lag.numel() != M):
        raise ValueError("lag: one int32 per marker")
    cap = M * (3 ** geom.ndim) if ghost > 0 else M
    idx = torch.empty(max(1, cap), dtype=torch.int32, device=X.device)
    xs = torch.empty((max(1, cap), geom.ndim), dtype=torch.float64, device=X.device)
    cells = torch.empty((max(1, cap), geom.ndim), dtype=torch.int32, device=X.device)
    check(ctx.lib.ibtk_le_index_set_box_list(ctx.h, ctypes.byref(geom.c), _ptr(X), _ptr(lag), M, ghost,
                                             pa[0] if pa else None, lo.p, hi.p, _ptr(idx), _ptr(xs), _ptr(cells), cap,
                                             ctypes.byref(cnt)))
    n = cnt.value
    return idx[:n].contiguous(), xs[:n].contiguous(), cells[:n].contiguous()


def list_in_box(ctx: Context, cells: torch.Tensor, indices: torch.Tensor, Xshift: Optional[torch.Tensor], box_lo,
                box_hi):
    """The entries of a cached list whose cell lies in [box_lo, box_hi], order kept
    (ibtk_le_list_in_box)."""
    n, nd = cells.shape
    lo, hi = _box_arg(box_lo, box_hi, nd)
    oi = torch.empty(max(1, n), dtype=torch.int32, device=cells.device)
    ox = torch.empty((max(1, n), nd), dtype=torch.float64, device=cells.device)
    cnt = ctypes.c_int(0)
    check(ctx.lib.ibtk_le_list_in_box(ctx.h, nd, _ptr(cells), _ptr(indices), _ptr(Xshift), n, lo.p, hi.p, _ptr(oi),
                                      _ptr(ox) if Xshift is not None else None, n, ctypes.byref(cnt)))
    k = cnt.value
    return oi[:k].contiguous(), (ox[:k].contiguous() if Xshift is not None else None)


def level_node_distribution(ctx: Context, geoms: Sequence[Geometry], dom_lo, dom_hi, X: torch.Tensor, ghost: int,
                            lag: Optional[torch.Tensor] = None, periodic=None):
    """LDataManager::computeNodeDistribution over the local patches of a level
    (ibtk_le_level_node_distribution): (order int32 device tensor, n_local, n_nonlocal);
    order[i] = the input index of node i, local nodes first."""
    M = X.shape[0]
    if lag is not None and (lag.dtype != torch.int32 or lag.numel() != M):
        raise ValueError("lag: one int32 per marker")
    nd = geoms[0].ndim
    lo, hi = _box_arg(dom_lo, dom_hi, nd)
    pa = _periodic_arg(periodic, nd)
    tab = (PatchGeom * len(geoms))(*[g.c for g in geoms])
    order = torch.empty(max(M, 1), dtype=torch.int32, device=X.device)
    nl, ng = ctypes.c_int(0), ctypes.c_int(0)
    check(ctx.lib.ibtk_le_level_node_distribution(ctx.h, len(geoms), tab, lo.p, hi.p, pa[0] if pa else None,
                                                  _ptr(X) if M else None, _ptr(lag), M, ghost,
                                                  _ptr(order), ctypes.byref(nl), ctypes.byref(ng)))
    return order[:nl.value + ng.value].contiguous(), nl.value, ng.value


def level_index_lists(ctx: Context, geoms: Sequence[Geometry], dom_lo, dom_hi, X: torch.Tensor, ghost: int,
                      periodic=None, order: str = "cells"):
    """LIndexSetData::cacheLocalIndices over every local patch of a level in one call
    (ibtk_le_level_index_lists): ((interior int32, None, offsets), (ghost-box int32, Xshift
    (n, ndim) float64, offsets)) -- the flat per-patch lists Level.from_flat and
    Level.select_interior take, offsets as Python lists of npatch + 1.  order "cells": a
    patch's entries in its box's cell order (the reference's); "markers": in marker order."""
    if order not in ("cells", "markers"):
        raise ValueError("order: 'cells' or 'markers'")
    M = X.shape[0]
    if M and (X.dtype != torch.float64 or not X.is_cuda or not X.is_contiguous()):
        raise ValueError("X: contiguous float64 device tensor")
    nd = geoms[0].ndim
    lo, hi = _box_arg(dom_lo, dom_hi, nd)
    pa = _periodic_arg(periodic, nd)
    P = len(geoms)
    tab = (PatchGeom * P)(*[g.c for g in geoms])
    ioff, goff = (ctypes.c_int * (P + 1))(), (ctypes.c_int * (P + 1))()
    icap, gcap = max(M, 1), max(M + M // 4, 1)
    for attempt in range(2):
        ii = torch.empty(icap, dtype=torch.int32, device=X.device)
        gi = torch.empty(gcap, dtype=torch.int32, device=X.device)
        gx = torch.empty((gcap, nd), dtype=torch.float64, device=X.device)
        rc = ctx.lib.ibtk_le_level_index_lists(ctx.h, P, tab, lo.p, hi.p, pa[0] if pa else None,
                                               _ptr(X) if M else None, M, ghost, 0 if order == "cells" else 1,
                                               _ptr(ii), icap,
                                               ctypes.cast(ioff, ctypes.c_void_p), _ptr(gi), _ptr(gx), gcap,
                                               ctypes.cast(goff, ctypes.c_void_p))
        if rc != 0 and attempt == 0 and (ioff[P] > icap or goff[P] > gcap):
            icap, gcap = max(icap, ioff[P]), max(gcap, goff[P])  # the sizes it reported
            continue
        check(rc)
        break
    ni, ng = ioff[P], goff[P]
    return ((ii[:ni].contiguous(), None, list(ioff)),
            (gi[:ng].contiguous(), gx[:ng].contiguous(), list(goff)))


def wrap_positions(ctx: Context, X: torch.Tensor, x_lower, x_upper, periodic=None):
    """beginDataRedistribution's periodic wrap of X (n, ndim) in place
    (ibtk_le_wrap_positions, LDataManager.cpp:1385-1399)."""
    if X.dtype != torch.float64 or not X.is_cuda or not X.is_contiguous() or X.dim() != 2:
        raise ValueError("X: contiguous (n, ndim) float64 device tensor")
    nd = X.shape[1]
    lo = (ctypes.c_double * nd)(*[float(v) for v in x_lower])
    hi = (ctypes.c_double * nd)(*[float(v) for v in x_upper])
    pa = _periodic_arg(periodic, nd)
    check(ctx.lib.ibtk_le_wrap_positions(ctx.h, nd, X.shape[0], _ptr(X), ctypes.cast(lo, ctypes.c_void_p),
                                         ctypes.cast(hi, ctypes.c_void_p), pa[0] if pa else None))
    return X


def ldata_reorder(ctx: Context, order: torch.Tensor, *arrays: torch.Tensor):
    """endDataRedistribution's reorder of LData arrays (ibtk_le_ldata_reorder): for each
    (M, ...) float64 device array, a new array whose row i is the old row order[i]."""
    outs = []
    for a in arrays:
        if a.dtype != torch.float64 or not a.is_cuda or not a.is_contiguous():
            raise ValueError("LData arrays: contiguous float64 device tensors")
        depth = a[0].numel() if a.shape[0] else 1
        out = torch.empty((order.numel(),) + tuple(a.shape[1:]), dtype=a.dtype, device=a.device)
        check(ctx.lib.ibtk_le_ldata_reorder(ctx.h, _ptr(order), order.numel(), _ptr(a), depth, _ptr(out)))
        outs.append(out)
    return outs


def node_distribution(ctx: Context, geom: Geometry, X: torch.Tensor, ghost: int, lag: Optional[torch.Tensor] = None):
    """LDataManager::computeNodeDistribution for one patch (ibtk_le_node_distribution):
    (order int32 device tensor, n_local, n_nonlocal)."""
    M = X.shape[0]
    if lag is not None and (lag.dtype != torch.int32 or lag.numel() != M):
        raise ValueError("lag: one int32 per marker")
    order = torch.empty(max(M, 1), dtype=torch.int32, device=X.device)
    nl, ng = ctypes.c_int(0), ctypes.c_int(0)
    check(ctx.lib.ibtk_le_node_distribution(ctx.h, ctypes.byref(geom.c), _ptr(X), _ptr(lag), M, ghost, _ptr(order),
                                            ctypes.byref(nl), ctypes.byref(ng)))
    return order[:nl.value + ng.value].contiguous(), nl.value, ng.value


def periodic_index_list(ctx: Context, geom: Geometry, X: torch.Tensor, ghost: int, periodic=None):
    """(indices int32, Xshift float64 [n, ndim]) device tensors, in the reference's
    order (ghost-box cells in iteration order, marker index within a cell)."""
    M = X.shape[0]
    cnt = ctypes.c_int(0)
    pa = _periodic_arg(periodic, geom.ndim)
    cap = M * (3 ** geom.ndim) if ghost > 0 else M
    idx = torch.empty(max(1, cap), dtype=torch.int32, device=X.device)
    xs = torch.empty((max(1, cap), geom.ndim), dtype=torch.float64, device=X.device)
    check(ctx.lib.ibtk_le_periodic_index_list(ctx.h, ctypes.byref(geom.c), _ptr(X), M, ghost,
                                              pa[0] if pa else None, _ptr(idx), _ptr(xs), cap, ctypes.byref(cnt)))
    n = cnt.value
    return idx[:n].contiguous(), xs[:n].contiguous()


def mark_stencils(ctx: Context, markers: Markers, kernel: str, centering: str, geom: Geometry, X: torch.Tensor,
                  q_depth: int = 1, axis: int = 0):
    """uint8 masks (one per component, shaped like the arrays) of the points some stencil touches."""
    masks = [torch.zeros(geom.array_shape(centering, c, q_depth), dtype=torch.uint8, device=X.device)
             for c in range(geom.ncomp(centering))]
    arr = (ctypes.c_void_p * len(masks))(*[m.data_ptr() for m in masks])
    check(ctx.lib.ibtk_le_mark_stencils(ctx.h, markers.h, kernel_id(kernel), CENTERING[centering], axis,
                                        ctypes.byref(geom.c), arr, q_depth, _ptr(X)))
    return masks
