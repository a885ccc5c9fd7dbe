"""GPU tests of the drop-in boundary: the Fortran-symbol shims (host memory, the
exact lagrangian_<k>_{interp,spread}{2,3}d_ signatures) and the C++ LEInteractor
facade.  Both are checked against the oracle / analytic identities.
"""
import ctypes
import subprocess
from pathlib import Path

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parents[1]


@pytest.fixture(scope="module")
def lib():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from ibamr_amd import _lib
    return _lib.load()


def _i(v):
    return ctypes.byref(ctypes.c_int(int(v)))


def _dp(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))


def _ip(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_int))


def call_shim(lib, op, kname, ndim, dx, xlo, ilo, ihi, g, u, idx, xs, X, V, depth=1, axis=None):
    f = getattr(lib, f"lagrangian_{kname}_{op}{ndim}d_")
    f.restype = None
    dxa, xla = np.ascontiguousarray(dx, float), np.ascontiguousarray(xlo, float)
    xua = xla + 1.0
    head = [_dp(dxa), _dp(xla), _dp(xua), _i(depth)]
    if kname == "discontinuous_linear":
        head.append(_i(axis or 0))
    box = []
    for d in range(ndim):
        box += [_i(ilo[d]), _i(ihi[d])]
    gc = [_i(g[d]) for d in range(ndim)]
    lst = [_ip(idx), _dp(xs), _i(idx.size)]
    if op == "interp":
        f(*head, *box, *gc, _dp(u), *lst, _dp(X), _dp(V))
    else:
        f(*head, *lst, _dp(X), _dp(V), *box, *gc, _dp(u))


KMAP = {"IB_4": "ib_4", "IB_6": "ib_6", "PIECEWISE_LINEAR": "piecewise_linear", "IB_4_W8": "ib_4_w8",
        "DISCONTINUOUS_LINEAR": "discontinuous_linear", "PIECEWISE_CUBIC": "piecewise_cubic", "IB_3": "ib_3",
        "PIECEWISE_CONSTANT": "piecewise_constant"}


@pytest.mark.parametrize("kernel", list(KMAP))
@pytest.mark.parametrize("ndim", [2, 3])
def test_fortran_shims_match_oracle(lib, oracle, kernel, ndim):
    rng = np.random.default_rng(17)
    g = oracle.min_ghost_width(kernel)
    ilo = [2, -3, 1][:ndim]
    ihi = [ilo[d] + 9 for d in range(ndim)]
    dx = [0.1] * ndim
    xlo = [0.2, -0.3, 0.0][:ndim]
    depth = 2
    shape = oracle.ghost_shape(ilo, ihi, [g] * ndim, depth)
    u = rng.uniform(-1, 1, shape)
    M = 120
    X = np.array(xlo) + rng.uniform(-0.05, 1.05, (M, ndim))
    idx = rng.integers(0, M, 150).astype(np.int32)  # duplicates on purpose
    xs = np.zeros((idx.size, ndim))
    # interp: the last entry of a repeated marker wins (Fortran l-loop order)
    V = np.full((M, depth), 7.0)
    call_shim(lib, "interp", KMAP[kernel], ndim, dx, xlo, ilo, ihi, [g] * ndim, u, idx, xs, X, V, depth, axis=1)
    Vo = np.full((M, depth), 7.0)
    oracle.interp(kernel, dx, xlo, ilo, ihi, [g] * ndim, u, idx, xs, X, Vo, depth=depth, axis=1)
    assert np.array_equal(V, Vo)
    # spread: same sums to rounding (the shim sums in canonical binned order)
    F = rng.uniform(-1, 1, (M, depth))
    ug = u.copy()
    call_shim(lib, "spread", KMAP[kernel], ndim, dx, xlo, ilo, ihi, [g] * ndim, ug, idx, xs, X, F, depth, axis=1)
    uo = u.copy()
    oracle.spread(kernel, dx, xlo, ilo, ihi, [g] * ndim, uo, idx, xs, X, F, depth=depth, axis=1)
    assert np.abs(ug - uo).max() <= 1e-12 * np.abs(uo).max()


def _facade_exe():
    exe = ROOT / "ibamr_amd" / "lib" / "facade_test"
    src = ROOT / "tests" / "cpp" / "facade_test.cpp"
    hdr = ROOT / "include" / "ibtk_le" / "LEInteractor.h"
    if not exe.exists() or exe.stat().st_mtime < max(src.stat().st_mtime, hdr.stat().st_mtime):
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O2", "-std=c++17", f"-I{ROOT / 'include'}",
                        str(src), f"-L{exe.parent}", "-libtk_le", "-Wl,-rpath,$ORIGIN", "-o", str(exe)], check=True)
    return exe


def test_cpp_facade(tmp_path):
    """Every overload form of the C++ facade (include/ibtk_le/LEInteractor.h: LData +
    index set, raw arrays + index set, std::vector and raw arrays with sizes, each on
    Cell / Node / Side / Edge data) against the oracle on one periodic 16^3 patch:
    interp of the index set's interior list, of its sub-box list (buildLocalIndices'
    box branch, LEInteractor.cpp:3070-3106, cells reaching into the ghost region) and
    of the markers whose cell is in a sub-box (some outside it) within 1e-13 (the two
    index-set forms and the two box forms bit for bit alike); spread of the ghost-box
    list (with periodic images), of the sub-box list and of the sub-box markers within
    1e-12 (LEInteractor.cpp:690-2397).  Then a patch with physical faces in x and z:
    too few ghosts throw (LEInteractor.cpp:2729-2745); with enough, spread + the
    adjoint physical fold (LDataManager.cpp:655-659) within 1e-12 of the oracle.  Form u:
    USER_DEFINED through LEInteractor::s_kernel_fcn (a 3-point kernel function) on the
    index set's lists, against the oracle's userDefinedInterpolate / Spread restatement."""
    from oracle import oracle as ora
    from test_gpu_parity import oracle_call

    from ibamr_amd.le import Geometry
    N, g, M, depth_c = 16, 3, 600, 2
    geom = Geometry.periodic_unit([N, N, N], g)
    rng = np.random.default_rng(17)
    X = rng.uniform(0.0, 1.0, (M, 3))
    X[:20] = np.floor(X[:20] * N) / N  # on cell faces
    F = rng.uniform(-1, 1, (M, 3))
    ii, xi, _ = ora.periodic_index_list(X, geom.x_lower, geom.x_upper, geom.dx, geom.ilower, geom.iupper, g,
                                        which="interior")
    ia, xa, ca = ora.periodic_index_list(X, geom.x_lower, geom.x_upper, geom.dx, geom.ilower, geom.iupper, g,
                                         which="all")
    sub = ([-2, 3, 1], [9, 17, 12])  # reaches below x and above y into the ghost cells
    sets = ora.lnode_set_data(X, geom.x_lower, geom.x_upper, geom.dx, geom.ilower, geom.iupper, g)
    ie, xe, _ = ora.build_local_indices(sets, geom.dx, geom.ilower, geom.iupper, g, sub)
    # the box forms: the markers whose cell is in the sub-box, no shifts (LEInteractor.cpp:3110-3139)
    cm = ora.get_cell_index(X, geom.x_lower, geom.x_upper, geom.dx, geom.ilower, geom.iupper)
    inb = np.all((cm >= np.array(sub[0])) & (cm <= np.array(sub[1])), axis=1)
    assert 0 < inb.sum() < M
    ib = np.nonzero(inb)[0].astype(np.int32)
    xb = np.zeros((ib.size, 3))
    # the physical-face patch: no images across x and z
    ip, xp, _ = ora.periodic_index_list(X, geom.x_lower, geom.x_upper, geom.dx, geom.ilower, geom.iupper, g,
                                        periodic=[False, True, False], which="all")
    u = {"cell": [rng.uniform(-1, 1, geom.array_shape("cell", 0, depth_c))],
         "node": [rng.uniform(-1, 1, geom.array_shape("node", 0, 1))],
         "side": [rng.uniform(-1, 1, geom.array_shape("side", a)) for a in range(3)],
         "edge": [rng.uniform(-1, 1, geom.array_shape("edge", a)) for a in range(3)]}
    (tmp_path / "meta.txt").write_text(f"{N} {g} {M} {ii.size} {ia.size} {depth_c}\n"
                                       f"{' '.join(map(str, sub[0]))} {' '.join(map(str, sub[1]))}\n")
    (tmp_path / "meta_phys.txt").write_text(f"{ip.size}\n")
    A = rng.uniform(0.2, 1.0, (3, 6))
    B = rng.uniform(0.2, 1.0, (3, 6))
    G = rng.uniform(-1, 1, (3, 6))
    for name, arr in [("X", X), ("F", F), ("idx_int", ii.astype(np.int32)), ("xs_int", xi),
                      ("idx_all", ia.astype(np.int32)), ("xs_all", xa), ("cells_all", ca.astype(np.int32)),
                      ("idx_phys", ip.astype(np.int32)), ("xs_phys", xp), ("bc_a", A), ("bc_b", B), ("bc_g", G),
                      ("u_cell", u["cell"][0]),
                      ("u_node", u["node"][0])] + [(f"u_side{a}", u["side"][a]) for a in range(3)] + \
            [(f"u_edge{a}", u["edge"][a]) for a in range(3)]:
        np.ascontiguousarray(arr).tofile(tmp_path / f"{name}.bin")
    r = subprocess.run([str(_facade_exe()), str(tmp_path)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "FACADE OK" in r.stdout, r.stdout + r.stderr
    for cent in ("cell", "node", "side", "edge"):
        depth = depth_c if cent == "cell" else 1
        Qd = 3 if cent in ("side", "edge") else depth
        nc = len(u[cent])
        Q = {f: np.fromfile(tmp_path / f"Q_{cent}_{f}.bin").reshape(M, Qd) for f in "abcde"}
        fs = {f: [np.fromfile(tmp_path / f"f_{cent}_{f}_{a}.bin").reshape(u[cent][a].shape) for a in range(nc)]
              for f in "abcde"}
        assert np.array_equal(Q["a"], Q["b"]) and np.array_equal(Q["c"], Q["d"]), cent
        for a in range(nc):
            assert np.array_equal(fs["a"][a], fs["b"][a]) and np.array_equal(fs["c"][a], fs["d"][a]), cent
        Sv = F[:, [k % 3 for k in range(Qd)]].copy()
        for form, (idx, xs) in (("a", (ii, xi)), ("c", (ib, xb)), ("e", (ie, xe))):
            Qo = np.full((M, Qd), -7.0)
            oracle_call(ora, "interp", "IB_4", cent, geom, [x.copy() for x in u[cent]], idx, xs, X, Qo, depth)
            scale = max(np.abs(Qo).max(), 1e-300)
            assert np.abs(Q[form] - Qo).max() <= 1e-13 * scale, f"{cent} {form} interp"
        for form, (idx, xs) in (("a", (ia, xa)), ("c", (ib, xb)), ("e", (ie, xe))):
            fo = [np.zeros_like(x) for x in u[cent]]
            oracle_call(ora, "spread", "IB_4", cent, geom, fo, idx, xs, X, Sv.copy(), depth)
            for a in range(nc):
                scale = max(np.abs(fo[a]).max(), 1e-300)
                assert np.abs(fs[form][a] - fo[a]).max() <= 1e-12 * scale, f"{cent} {form} spread comp {a}"
    # form u: USER_DEFINED through LEInteractor::s_kernel_fcn (facade_test.cpp's user_phi3)
    from test_gpu_user import phi3
    ora.set_user_kernel(phi3, 3)
    try:
        for cent in ("cell", "node", "side", "edge"):
            depth = depth_c if cent == "cell" else 1
            Qd = 3 if cent in ("side", "edge") else depth
            nc = len(u[cent])
            Qg = np.fromfile(tmp_path / f"Q_{cent}_u.bin").reshape(M, Qd)
            Qo = np.full((M, Qd), -7.0)
            oracle_call(ora, "interp", "USER_DEFINED", cent, geom, [x.copy() for x in u[cent]], ii, xi, X, Qo, depth)
            assert np.abs(Qg - Qo).max() <= 1e-13 * max(np.abs(Qo).max(), 1e-300), f"{cent} user interp"
            Sv = F[:, [k % 3 for k in range(Qd)]].copy()
            fo = [np.zeros_like(x) for x in u[cent]]
            oracle_call(ora, "spread", "USER_DEFINED", cent, geom, fo, ia, xa, X, Sv, depth)
            for a in range(nc):
                fg = np.fromfile(tmp_path / f"f_{cent}_u_{a}.bin").reshape(fo[a].shape)
                assert np.abs(fg - fo[a]).max() <= 1e-12 * max(np.abs(fo[a]).max(), 1e-300), f"{cent} user spread {a}"
    finally:
        ora.set_user_kernel(None, 4)
    # the physical-face patch: spread of its list, then the adjoint fold of x and z
    fo = [np.zeros(geom.array_shape("side", a)) for a in range(3)]
    oracle_call(ora, "spread", "IB_4", "side", geom, fo, ip, xp, X, F.copy(), 1)
    ora.phys_bdry_side(geom.ilower, geom.iupper, g, geom.dx, fo, [1, 1, 0, 0, 1, 1], A, B, G, adjoint=True)
    for a in range(3):
        fg = np.fromfile(tmp_path / f"f_phys_{a}.bin").reshape(fo[a].shape)
        scale = max(np.abs(fo[a]).max(), 1e-300)
        assert np.abs(fg - fo[a]).max() <= 1e-12 * scale, f"physical faces: spread + fold, comp {a}"
