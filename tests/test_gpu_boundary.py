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


def test_cpp_facade():
    exe = ROOT / "ibamr_amd" / "lib" / "facade_test"
    src = ROOT / "tests" / "cpp" / "facade_test.cpp"
    if not exe.exists() or exe.stat().st_mtime < src.stat().st_mtime:
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O2", "-std=c++17", f"-I{ROOT / 'include'}",
                        str(src), f"-L{exe.parent}", "-libtk_le", "-Wl,-rpath,$ORIGIN", "-o", str(exe)], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "FACADE OK" in r.stdout, r.stdout + r.stderr
