"""CPU oracle for the LE-coupling hot path -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this module, and only as the checker (or the timed CPU
baseline).  The product path (``ibamr_amd``) never imports it.

Parity status: **parity unpinned** against the reference binary (the Fortran
needs m4 + SAMRAI's ``pdat_m4arrdim*.i``, both absent).
The arithmetic lives in ``le_oracle.c`` (a restatement of
``ibtk/src/lagrangian/fortran/lagrangian_interaction{2,3}d.f.m4``); this module
adds ctypes bindings and restates the C++ wrappers around it:

* ``side_interp`` / ``side_spread`` -- ``LEInteractor.cpp:1017-1053`` and
  ``:1876-1911`` (per-axis call, ``x_lower[axis] -= dx/2``,
  ``SideGeometry::toSideBox``, AoS<->SoA of Q).
* ``cell_*`` -- ``LEInteractor.cpp:708-755`` / ``1548-1613``.
* ``node_*`` -- ``LEInteractor.cpp:838-967`` (``x_lower -= dx/2`` all dims,
  ``toNodeBox``).
* ``periodic_index_list`` -- ``LIndexSetData::cacheLocalIndices``
  (``LIndexSetData.cpp:83-169``) for one patch covering a periodic domain,
  with ``IndexUtilities::getCellIndex`` (``IndexUtilities-inl.h:66-89``).
* ``lnode_set_data`` / ``build_local_indices`` -- the patch's per-cell node sets
  and ``LEInteractor::buildLocalIndices`` over them for any box
  (``LEInteractor.cpp:3031-3108``), offsets from the cells (an independent
  restatement of the lists ``periodic_index_list`` builds from the images).
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path

import numpy as np

_HERE = Path(__file__).resolve().parent
_LIB_PATH = _HERE / "build" / "libleoracle.so"

KERNELS = {
    "PIECEWISE_CONSTANT": 0,
    "DISCONTINUOUS_LINEAR": 1,
    "PIECEWISE_LINEAR": 2,
    "PIECEWISE_CUBIC": 3,
    "IB_3": 4,
    "IB_4": 5,
    "IB_4_W8": 6,
    "IB_6": 7,
    "BSPLINE_4": 8,
}
STENCIL = {"PIECEWISE_CONSTANT": 1, "DISCONTINUOUS_LINEAR": 2, "PIECEWISE_LINEAR": 2, "PIECEWISE_CUBIC": 4,
           "IB_3": 4, "IB_4": 4, "IB_4_W8": 8, "IB_6": 6, "BSPLINE_4": 4}

_lib = None


def build():
    """Compile le_oracle.c with the committed Makefile (gcc, -ffp-contract=off)."""
    import subprocess
    subprocess.run(["make", "-s", "-C", str(_HERE)], check=True)


def lib():
    global _lib
    if _lib is None:
        if not _LIB_PATH.exists():
            build()
        L = ctypes.CDLL(str(_LIB_PATH))
        dp = ctypes.POINTER(ctypes.c_double)
        ip = ctypes.POINTER(ctypes.c_int)
        c_int = ctypes.c_int
        for name in ("ora_interp", "ora_spread"):
            f = getattr(L, name)
            f.restype = c_int
            f.argtypes = [c_int, c_int, dp, dp, c_int, c_int, ip, ip, ip, dp, ip, dp, c_int, dp, dp]
        L.ora_closed_form_weights.restype = c_int
        L.ora_closed_form_weights.argtypes = [c_int, ctypes.c_double, c_int, dp]
        L.ora_lagrangian_floor.restype = c_int
        L.ora_lagrangian_floor.argtypes = [ctypes.c_double]
        L.ora_ib_3_delta.restype = ctypes.c_double
        L.ora_ib_3_delta.argtypes = [ctypes.c_double]
        L.ora_piecewise_cubic_delta.restype = ctypes.c_double
        L.ora_piecewise_cubic_delta.argtypes = [ctypes.c_double]
        L.ora_user_call.restype = c_int
        L.ora_user_call.argtypes = [ctypes.c_void_p, c_int, c_int, c_int, dp, dp, c_int, ip, ip, ip, dp, ip, dp, c_int,
                                    dp, dp]
        L.ora_phys_bdry_side.restype = c_int
        L.ora_phys_bdry_side.argtypes = [c_int, ip, ip, c_int, dp, dp, dp, dp, ip, dp, dp, dp, c_int]
        _lib = L
    return _lib


def _dp(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))


def _ip(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_int))


def _f64(a):
    return np.ascontiguousarray(a, dtype=np.float64)


def _i32(a):
    return np.ascontiguousarray(a, dtype=np.int32)


# USER_DEFINED: LEInteractor::s_kernel_fcn / s_kernel_fcn_stencil_size (LEInteractor.cpp:651-652),
# IB_4's ib4_kernel_fcn (:629-648) and 4 by default
def ib4_kernel_fcn(r):
    r = abs(r)
    if r < 1.0:
        t2 = r * r
        t6 = np.sqrt(-0.4e1 * t2 + 0.4e1 * r + 0.1e1)
        return -r / 0.4e1 + 0.3e1 / 0.8e1 + t6 / 0.8e1
    if r < 2.0:
        t2 = r * r
        t6 = np.sqrt(0.12e2 * r - 0.7e1 - 0.4e1 * t2)
        return -r / 0.4e1 + 0.5e1 / 0.8e1 - t6 / 0.8e1
    return 0.0


_USER_FN = ctypes.CFUNCTYPE(ctypes.c_double, ctypes.c_double)
_user = {"fn": ib4_kernel_fcn, "S": 4, "cb": _USER_FN(ib4_kernel_fcn)}


def set_user_kernel(fn, stencil_size):
    """LEInteractor::s_kernel_fcn = fn; s_kernel_fcn_stencil_size = stencil_size (None: the default)."""
    fn = fn if fn is not None else ib4_kernel_fcn
    _user.update(fn=fn, S=int(stencil_size), cb=_USER_FN(fn))
    STENCIL["USER_DEFINED"] = int(stencil_size)


STENCIL["USER_DEFINED"] = 4


def _user_call(spread_, dx, x_lower, ilower, iupper, nugc, u, indices, Xshift, X, V, depth):
    ndim = len(ilower)
    idx, xs, X = _i32(indices), _f64(Xshift), _f64(X)
    rc = lib().ora_user_call(ctypes.cast(_user["cb"], ctypes.c_void_p), _user["S"], int(spread_), ndim, _dp(_f64(dx)),
                             _dp(_f64(x_lower)), int(depth), _ip(_i32(ilower)), _ip(_i32(iupper)), _ip(_i32(nugc)),
                             _dp(u), _ip(idx), _dp(xs), int(idx.size), _dp(X), _dp(V))
    if rc != 0:
        raise RuntimeError(f"ora_user_call failed ({rc})")


def kernel_id(kernel):
    if kernel not in KERNELS:
        raise ValueError(f"unknown kernel function {kernel}")
    return KERNELS[kernel]


def min_ghost_width(kernel):
    """LEInteractor::getMinimumGhostWidth, LEInteractor.cpp:684-687."""
    return STENCIL[kernel] // 2 + 1


def weights_1d(kernel, X_o_dx, ilower=0):
    """1-D weights of a closed-form kernel: (ic_lower, w[W])."""
    W = STENCIL[kernel]
    w = np.zeros(8)
    icl = lib().ora_closed_form_weights(kernel_id(kernel), float(X_o_dx), int(ilower), _dp(w))
    return icl, w[:W].copy()


# --------------------------------------------------------------------------
# raw Fortran-call equivalents
# --------------------------------------------------------------------------
def ghost_shape(ilower, iupper, nugc, depth=1):
    """numpy shape (C order) of the Fortran array u(CELLdVECG, 0:depth-1)."""
    n = [iupper[d] - ilower[d] + 1 + 2 * nugc[d] for d in range(len(ilower))]
    return (depth,) + tuple(reversed(n))


def interp(kernel, dx, x_lower, ilower, iupper, nugc, u, indices, Xshift, X, V, depth=1, axis=0):
    """One call of lagrangian_<kernel>_interp{2,3}d_ (writes V in place); USER_DEFINED:
    LEInteractor::userDefinedInterpolate."""
    ndim = len(ilower)
    u = _f64(u)
    assert u.size == int(np.prod(ghost_shape(ilower, iupper, nugc, depth)))
    if kernel == "USER_DEFINED":
        assert V.dtype == np.float64 and V.flags.c_contiguous
        _user_call(False, dx, x_lower, ilower, iupper, nugc, u, indices, Xshift, X, V, depth)
        return V
    idx, xs, X = _i32(indices), _f64(Xshift), _f64(X)
    assert V.dtype == np.float64 and V.flags.c_contiguous
    rc = lib().ora_interp(kernel_id(kernel), ndim, _dp(_f64(dx)), _dp(_f64(x_lower)), int(depth), int(axis),
                          _ip(_i32(ilower)), _ip(_i32(iupper)), _ip(_i32(nugc)), _dp(u), _ip(idx), _dp(xs),
                          int(idx.size), _dp(X), _dp(V))
    if rc != 0:
        raise RuntimeError(f"ora_interp failed ({rc})")
    return V


def spread(kernel, dx, x_lower, ilower, iupper, nugc, u, indices, Xshift, X, V, depth=1, axis=0):
    """One call of lagrangian_<kernel>_spread{2,3}d_ (accumulates into u); USER_DEFINED:
    LEInteractor::userDefinedSpread."""
    ndim = len(ilower)
    assert u.dtype == np.float64 and u.flags.c_contiguous
    assert u.size == int(np.prod(ghost_shape(ilower, iupper, nugc, depth)))
    if kernel == "USER_DEFINED":
        _user_call(True, dx, x_lower, ilower, iupper, nugc, u, indices, Xshift, X, _f64(V), depth)
        return u
    idx, xs, X, V = _i32(indices), _f64(Xshift), _f64(X), _f64(V)
    rc = lib().ora_spread(kernel_id(kernel), ndim, _dp(_f64(dx)), _dp(_f64(x_lower)), int(depth), int(axis),
                          _ip(_i32(ilower)), _ip(_i32(iupper)), _ip(_i32(nugc)), _dp(u), _ip(idx), _dp(xs),
                          int(idx.size), _dp(X), _dp(V))
    if rc != 0:
        raise RuntimeError(f"ora_spread failed ({rc})")
    return u


# --------------------------------------------------------------------------
# C++ wrapper restatements
# --------------------------------------------------------------------------
def side_box(box_lo, box_hi, axis):
    """SideGeometry::toSideBox: upper[axis] + 1."""
    hi = list(box_hi)
    hi[axis] += 1
    return list(box_lo), hi


def side_interp(kernel, dx, x_lower, box_lo, box_hi, gcw, u_axes, indices, Xshift, X, Q):
    """LEInteractor::interpolate on SideData (LEInteractor.cpp:1017-1053).

    u_axes[a] is the ghosted side array of axis a; Q is AoS (M, NDIM), written
    at the listed markers only.
    """
    ndim = len(box_lo)
    idx = _i32(indices)
    if idx.size == 0:
        return Q
    local_sz = int(idx.max()) + 1
    for axis in range(ndim):
        xl = [float(v) for v in x_lower]
        xl[axis] -= 0.5 * dx[axis]
        lo, hi = side_box(box_lo, box_hi, axis)
        Qa = np.zeros(local_sz)
        interp(kernel, dx, xl, lo, hi, gcw, u_axes[axis], idx, Xshift, X, Qa, depth=1, axis=axis)
        Q.reshape(-1, ndim)[idx, axis] = Qa[idx]
    return Q


def side_spread(kernel, dx, x_lower, box_lo, box_hi, gcw, u_axes, indices, Xshift, X, Q):
    """LEInteractor::spread on SideData (LEInteractor.cpp:1876-1911)."""
    ndim = len(box_lo)
    idx = _i32(indices)
    if idx.size == 0:
        return u_axes
    local_sz = int(idx.max()) + 1
    Qr = np.asarray(Q).reshape(-1, ndim)
    for axis in range(ndim):
        xl = [float(v) for v in x_lower]
        xl[axis] -= 0.5 * dx[axis]
        lo, hi = side_box(box_lo, box_hi, axis)
        Qa = np.zeros(local_sz)
        Qa[idx] = Qr[idx, axis]
        spread(kernel, dx, xl, lo, hi, gcw, u_axes[axis], idx, Xshift, X, Qa, depth=1, axis=axis)
    return u_axes


def cell_interp(kernel, dx, x_lower, box_lo, box_hi, gcw, u, indices, Xshift, X, Q, depth):
    """LEInteractor::interpolate on CellData (LEInteractor.cpp:1058-1146 -> private :2399)."""
    return interp(kernel, dx, x_lower, box_lo, box_hi, gcw, u, indices, Xshift, X, Q, depth=depth)


def cell_spread(kernel, dx, x_lower, box_lo, box_hi, gcw, u, indices, Xshift, X, Q, depth):
    return spread(kernel, dx, x_lower, box_lo, box_hi, gcw, u, indices, Xshift, X, Q, depth=depth)


def node_interp(kernel, dx, x_lower, box_lo, box_hi, gcw, u, indices, Xshift, X, Q, depth):
    """NodeData: x_lower -= dx/2 in every dim, NodeGeometry::toNodeBox (upper + 1)."""
    xl = [x_lower[d] - 0.5 * dx[d] for d in range(len(box_lo))]
    hi = [h + 1 for h in box_hi]
    return interp(kernel, dx, xl, box_lo, hi, gcw, u, indices, Xshift, X, Q, depth=depth)


def node_spread(kernel, dx, x_lower, box_lo, box_hi, gcw, u, indices, Xshift, X, Q, depth):
    xl = [x_lower[d] - 0.5 * dx[d] for d in range(len(box_lo))]
    hi = [h + 1 for h in box_hi]
    return spread(kernel, dx, xl, box_lo, hi, gcw, u, indices, Xshift, X, Q, depth=depth)


def get_cell_index(X, x_lower, x_upper, dx, ilower, iupper):
    """IndexUtilities::getCellIndex (IndexUtilities-inl.h:66-89), vectorised."""
    X = np.asarray(X, dtype=np.float64)
    ndim = X.shape[1]
    out = np.empty(X.shape, dtype=np.int64)
    for d in range(ndim):
        dl = X[:, d] - x_lower[d]
        du = X[:, d] - x_upper[d]
        lower = np.abs(dl) <= np.abs(du)
        out[:, d] = np.where(lower, ilower[d] + np.floor(dl / dx[d]), iupper[d] + np.floor(du / dx[d]) + 1)
    return out


def periodic_index_list(X, x_lower, x_upper, dx, box_lo, box_hi, ghost, periodic=None, lag=None, which="all"):
    """(indices, Xshift, cells) for one patch covering a periodic domain.

    Every marker appears once at its own cell (interior) and once per periodic
    image whose cell falls in the ghost box, with Xshift = +/-L in the
    wrapped dims -- the lists LIndexSetData::cacheLocalIndices builds
    (LIndexSetData.cpp:111-166: offset = -periodic_shift below the patch,
    +periodic_shift above it).  Order: the ghost box's cells in iteration order
    (x fastest), within a cell by Lagrangian index (lag[s]; the marker index s
    when lag is None) -- the LNodeSet order after LDataManager.cpp:1487-1493's
    sort.  which: "all" (d_local_petsc_indices), "interior" (cells in the patch
    box, d_interior_*) or "ghost" (the others, d_ghost_*), LIndexSetData.cpp:143-165.
    """
    X = np.asarray(X, dtype=np.float64)
    M, ndim = X.shape
    periodic = [True] * ndim if periodic is None else periodic
    N = [box_hi[d] - box_lo[d] + 1 for d in range(ndim)]
    cells = get_cell_index(X, x_lower, x_upper, dx, box_lo, box_hi)
    # the patch's own markers: beginDataRedistribution keeps a marker in the patch
    # whose box holds its cell (LDataManager.cpp:1457-1482); the ghost cells get
    # the periodic images of those
    own = np.ones(M, dtype=bool)
    for d in range(ndim):
        own &= (cells[:, d] >= box_lo[d]) & (cells[:, d] <= box_hi[d])
    ids = np.nonzero(own)[0]
    cells = cells[ids]
    M = ids.size
    ents_s, ents_off, ents_cell = [ids], [np.zeros((M, ndim), np.int64)], [cells]
    # images: shift the cell by -N (image below) or +N (image above) per dim
    import itertools
    for shifts in itertools.product(*[(-1, 0, 1) if periodic[d] else (0,) for d in range(ndim)]):
        if all(s == 0 for s in shifts):
            continue
        c = cells.copy()
        for d in range(ndim):
            c[:, d] += shifts[d] * N[d]
        inside = np.ones(M, dtype=bool)
        for d in range(ndim):
            inside &= (c[:, d] >= box_lo[d] - ghost) & (c[:, d] <= box_hi[d] + ghost)
        if inside.any():
            sel = np.nonzero(inside)[0]
            ents_s.append(ids[sel])
            ents_off.append(np.tile(np.array(shifts, np.int64) * np.array(N), (sel.size, 1)))
            ents_cell.append(c[sel])
    s = np.concatenate(ents_s)
    off = np.concatenate(ents_off)
    cell = np.concatenate(ents_cell)
    # cell-major order (x fastest) then Lagrangian index: the IndexData iteration order
    key = np.zeros(s.size, dtype=np.int64)
    stride = 1
    interior = np.ones(s.size, dtype=bool)
    for d in range(ndim):
        key += (cell[:, d] - (box_lo[d] - ghost)) * stride
        stride *= N[d] + 2 * ghost
        interior &= (cell[:, d] >= box_lo[d]) & (cell[:, d] <= box_hi[d])
    sel = {"all": np.ones(s.size, dtype=bool), "interior": interior, "ghost": ~interior}[which]
    s, off, cell, key = s[sel], off[sel], cell[sel], key[sel]
    lagv = s if lag is None else np.asarray(lag)[s]
    order = np.lexsort((s, lagv, key))
    # each cell's LNodeSet is uniqued by Lagrangian index (LDataManager.cpp:1487-1493;
    # of equal ones the lowest marker index is kept -- the reference's std::sort leaves
    # it unspecified)
    ks, ls = key[order], lagv[order]
    keep = np.ones(order.size, dtype=bool)
    keep[1:] = (ks[1:] != ks[:-1]) | (ls[1:] != ls[:-1])
    order = order[keep]
    Xshift = off[order].astype(np.float64) * np.asarray(dx)[None, :]
    return s[order].astype(np.int32), Xshift, cell[order]


def lnode_set_data(X, x_lower, x_upper, dx, box_lo, box_hi, ghost, periodic=None, lag=None):
    """The patch's LNodeSetData over its ghost box for one patch covering a periodic
    domain: {cell: [marker, ...]}.  A marker sits in the set of its getCellIndex cell
    (beginDataRedistribution keeps the patch box's markers, LDataManager.cpp:1446-1482),
    the ghost cells hold the periodic images of the patch's own cells (the index data's
    periodic ghost fill); each set sorted by Lagrangian index and uniqued
    (LDataManager.cpp:1487-1493, lowest marker index kept among equal ones)."""
    import itertools
    X = np.asarray(X, dtype=np.float64)
    M, ndim = X.shape
    periodic = [True] * ndim if periodic is None else periodic
    lagv = np.arange(M) if lag is None else np.asarray(lag, dtype=np.int64)
    N = [box_hi[d] - box_lo[d] + 1 for d in range(ndim)]
    c = get_cell_index(X, x_lower, x_upper, dx, box_lo, box_hi)
    sets = {}
    for m in range(M):
        if not all(box_lo[d] <= c[m, d] <= box_hi[d] for d in range(ndim)):
            continue
        for sh in itertools.product(*[(-1, 0, 1) if periodic[d] else (0,) for d in range(ndim)]):
            ci = tuple(int(c[m, d] + sh[d] * N[d]) for d in range(ndim))
            if all(box_lo[d] - ghost <= ci[d] <= box_hi[d] + ghost for d in range(ndim)):
                sets.setdefault(ci, []).append(m)
    for ci, lst in sets.items():
        lst.sort(key=lambda m: (lagv[m], m))
        out = []
        for m in lst:
            if not out or lagv[out[-1]] != lagv[m]:
                out.append(m)
        sets[ci] = out
    return sets


def build_local_indices(sets, dx, box_lo, box_hi, ghost, box, periodic=None):
    """LEInteractor::buildLocalIndices (LEInteractor.cpp:3031-3108) over an index set
    ``sets`` (lnode_set_data) of the patch [box_lo, box_hi] with `ghost` ghost cells, for
    any ``box`` = (lower, upper): the set's cells are walked in IndexData order (the
    ghost box's cells, x fastest), cells outside ``box`` skipped (:3075), and every node
    of a cell gets offset[d] = -periodic_shift(d) where the patch touches its lower
    periodic boundary in d and i(d) < ilower(d), +periodic_shift(d) where it touches
    the upper one and i(d) > iupper(d), else 0 (:3077-3093); Xshift = offset * dx (:3100).
    One patch covering the domain: it touches both periodic boundaries of every periodic
    dim and periodic_shift(d) = its cell count.  (box == the patch box / ghost box: the
    cached interior / all lists of cacheLocalIndices, LIndexSetData.cpp:111-166, which
    apply the same per-cell offsets -- :3061-3069.)  Returns (indices, Xshift, cells)."""
    import itertools
    ndim = len(box_lo)
    periodic = [True] * ndim if periodic is None else periodic
    N = [box_hi[d] - box_lo[d] + 1 for d in range(ndim)]
    blo, bhi = box
    idx, xs, cells = [], [], []
    ranges = [range(box_lo[d] - ghost, box_hi[d] + ghost + 1) for d in range(ndim)]
    for ci_rev in itertools.product(*reversed(ranges)):  # x fastest
        ci = tuple(reversed(ci_rev))
        if ci not in sets:
            continue
        if not all(blo[d] <= ci[d] <= bhi[d] for d in range(ndim)):
            continue
        off = [0] * ndim
        for d in range(ndim):
            if periodic[d] and ci[d] < box_lo[d]:
                off[d] = -N[d]
            elif periodic[d] and ci[d] > box_hi[d]:
                off[d] = +N[d]
        for m in sets[ci]:
            idx.append(m)
            xs.append([off[d] * dx[d] for d in range(ndim)])
            cells.append(list(ci))
    return (np.array(idx, dtype=np.int32), np.array(xs, dtype=np.float64).reshape(-1, ndim),
            np.array(cells, dtype=np.int64).reshape(-1, ndim))


def node_distribution(X, x_lower, x_upper, dx, box_lo, box_hi, ghost, lag=None):
    """LDataManager::computeNodeDistribution (LDataManager.cpp:2874-2947) for one
    patch: (order, n_local, n_nonlocal).  Local nodes (getCellIndex cell in the
    patch box) in box order (x fastest), each cell's LNodeSet sorted by Lagrangian
    index and uniqued (LDataManager.cpp:1487-1493); then the nonlocal nodes of the
    ghost cells (ghost-box order, same within-cell rule); markers beyond the ghost
    box are not numbered.  order[i] = input index of the node numbered i."""
    X = np.asarray(X, dtype=np.float64)
    M, ndim = X.shape
    lagv = np.arange(M) if lag is None else np.asarray(lag, dtype=np.int64)
    c = get_cell_index(X, x_lower, x_upper, dx, box_lo, box_hi)
    N = [box_hi[d] - box_lo[d] + 1 for d in range(ndim)]
    inside = np.ones(M, dtype=bool)
    ing = np.ones(M, dtype=bool)
    kin = np.zeros(M, dtype=np.int64)
    kg = np.zeros(M, dtype=np.int64)
    si = sg = 1
    for d in range(ndim):
        inside &= (c[:, d] >= box_lo[d]) & (c[:, d] <= box_hi[d])
        ing &= (c[:, d] >= box_lo[d] - ghost) & (c[:, d] <= box_hi[d] + ghost)
        kin += (c[:, d] - box_lo[d]) * si
        kg += (c[:, d] - (box_lo[d] - ghost)) * sg
        si *= N[d]
        sg *= N[d] + 2 * ghost
    key = np.where(inside, kin, np.where(ing, si + kg, np.iinfo(np.int64).max))
    order = np.lexsort((np.arange(M), lagv, key))
    ks, ls = key[order], lagv[order]
    keep = np.ones(M, dtype=bool)
    keep[1:] = (ks[1:] != ks[:-1]) | (ls[1:] != ls[:-1])
    keep &= ks != np.iinfo(np.int64).max
    order = order[keep]
    n_local = int((key[order] < si).sum())
    return order.astype(np.int32), n_local, int(order.size - n_local)


def level_node_distribution(X, lag, patches, dom_lo, dom_hi, x_lower, dx, ghost, periodic=None):
    """LDataManager::computeNodeDistribution (LDataManager.cpp:2874-2947) over the local
    patches of a level, written as the reference's loops (small cases only).

    patches: [(lo, hi)] cell boxes in PatchLevel order; the domain [dom_lo, dom_hi] with
    lower corner x_lower and spacing dx (cells by getCellIndex in that frame), periodic
    in the dims ``periodic[d]``.  Each patch's LNodeSetData holds, for every cell of its
    ghost box, the markers whose cell is that cell or -- across a periodic side -- whose
    image is, each set sorted by Lagrangian index and uniqued (LDataManager.cpp:
    1487-1493; lowest marker index kept).  Local loop (:2876-2892): patches in order,
    data_begin(patch_box) -- box cells, x fastest -- every node a new local index.
    Nonlocal loop (:2914-2944): patches in order, the ghost box minus the patch box
    walked in box order (SAMRAI's removeIntersections box-list order is not vendored:
    parity unpinned for that order), a node whose Lagrangian index has no index yet gets
    the next one.  Returns (order, n_local, n_nonlocal): order[i] = marker of node i."""
    import itertools
    X = np.asarray(X, dtype=np.float64)
    M, ndim = X.shape
    lagv = np.arange(M) if lag is None else np.asarray(lag, dtype=np.int64)
    periodic = [True] * ndim if periodic is None else periodic
    D = [dom_hi[d] - dom_lo[d] + 1 for d in range(ndim)]
    x_upper = [x_lower[d] + D[d] * dx[d] for d in range(ndim)]
    c = get_cell_index(X, x_lower, x_upper, dx, dom_lo, dom_hi)

    def cells_of(lo, hi):  # box order, x fastest
        for ci_rev in itertools.product(*[range(lo[d], hi[d] + 1) for d in reversed(range(ndim))]):
            yield tuple(reversed(ci_rev))

    def set_data(lo, hi):
        glo = [lo[d] - ghost for d in range(ndim)]
        ghi = [hi[d] + ghost for d in range(ndim)]
        sets = {}
        for m in range(M):
            for sh in itertools.product(*[(-1, 0, 1) if periodic[d] else (0,) for d in range(ndim)]):
                ci = tuple(int(c[m, d] + sh[d] * D[d]) for d in range(ndim))
                if all(glo[d] <= ci[d] <= ghi[d] for d in range(ndim)):
                    sets.setdefault(ci, []).append(m)
        for ci, lst in sets.items():
            lst.sort(key=lambda m: (lagv[m], m))
            out = []
            for m in lst:
                if not out or lagv[out[-1]] != lagv[m]:
                    out.append(m)
            sets[ci] = out
        return sets

    data = [set_data(lo, hi) for lo, hi in patches]
    order, seen = [], {}
    for (lo, hi), sets in zip(patches, data):
        for ci in cells_of(lo, hi):
            for m in sets.get(ci, []):
                seen[lagv[m]] = len(order)
                order.append(m)
    n_local = len(order)
    for (lo, hi), sets in zip(patches, data):
        glo = [lo[d] - ghost for d in range(ndim)]
        ghi = [hi[d] + ghost for d in range(ndim)]
        for ci in cells_of(glo, ghi):
            if all(lo[d] <= ci[d] <= hi[d] for d in range(ndim)):
                continue
            for m in sets.get(ci, []):
                if lagv[m] not in seen:
                    seen[lagv[m]] = len(order)
                    order.append(m)
    return np.array(order, dtype=np.int32), n_local, len(order) - n_local


# --------------------------------------------------------------------------
# physical-boundary operators (le_bdry_oracle.c)
# --------------------------------------------------------------------------
def side_ghost_shape(box_lo, box_hi, gcw, axis):
    """numpy shape (C order) of the ghosted side array of `axis` (uniform gcw)."""
    lo, hi = side_box(box_lo, box_hi, axis)
    return ghost_shape(lo, hi, [gcw] * len(box_lo))[1:]


def phys_bdry_side(box_lo, box_hi, gcw, dx, u_axes, phys, acoef, bcoef, gcoef, adjoint):
    """CartSideRobinPhysBdryOp on one patch of side data (in place).

    adjoint=False: setPhysicalBoundaryConditions (CartSideRobinPhysBdryOp.cpp:358-422);
    adjoint=True: accumulateFromPhysicalBoundaryData (:429-493).  phys[2d+upper]
    flags a physical face; acoef/bcoef/gcoef have shape (ndim, 2 ndim):
    [component axis, face location]."""
    ndim = len(box_lo)
    us = []
    for a in range(ndim):
        u = u_axes[a]
        assert u.dtype == np.float64 and u.flags.c_contiguous
        assert u.shape == side_ghost_shape(box_lo, box_hi, gcw, a)
        us.append(u)
    dummy = np.zeros(1)
    while len(us) < 3:
        us.append(dummy)
    A, B, G = (_f64(np.broadcast_to(np.asarray(c, np.float64), (ndim, 2 * ndim))) for c in (acoef, bcoef, gcoef))
    rc = lib().ora_phys_bdry_side(ndim, _ip(_i32(box_lo)), _ip(_i32(box_hi)), int(gcw), _dp(_f64(dx)), _dp(us[0]),
                                  _dp(us[1]), _dp(us[2]), _ip(_i32(phys)), _dp(A), _dp(B), _dp(G), int(adjoint))
    if rc != 0:
        raise RuntimeError(f"ora_phys_bdry_side failed ({rc})")
    return u_axes
