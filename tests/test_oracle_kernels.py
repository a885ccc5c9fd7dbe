"""CPU tests of the oracle (the restatement of the reference Fortran kernels).

Pins the restatement with (1) known-answer weights computed in 60-digit decimal
from the reference's own 1-D delta functions (tests/golden/kernel_weights.json,
made by tests/golden/make_golden.py) and (2) the analytic identities the
kernels are built to satisfy.  The reference has no test suite
of its own for this path, and its Fortran cannot be built here, so the oracle
is "parity unpinned" against the reference binary.
"""
import json
from decimal import Decimal
from pathlib import Path

import numpy as np
import pytest

GOLDEN = json.loads((Path(__file__).parent / "golden" / "kernel_weights.json").read_text())
ALL = ["PIECEWISE_CONSTANT", "DISCONTINUOUS_LINEAR", "PIECEWISE_LINEAR", "PIECEWISE_CUBIC", "IB_3", "IB_4",
       "IB_4_W8", "IB_6", "BSPLINE_4"]
SMOOTH = ["PIECEWISE_LINEAR", "PIECEWISE_CUBIC", "IB_3", "IB_4", "IB_4_W8", "IB_6", "BSPLINE_4"]


@pytest.mark.parametrize("case", [c for c in GOLDEN["cases"] if c["kernel"] in ("IB_4", "BSPLINE_4", "IB_4_W8", "IB_6")],
                         ids=lambda c: f"{c['kernel']}@{c['X_o_dx']}")
def test_closed_form_weights_known_answer(oracle, case):
    icl, w = oracle.weights_1d(case["kernel"], float(case["X_o_dx"]))
    assert icl == case["ic_lower"]
    expect = np.array([float(Decimal(v)) for v in case["w"]])
    np.testing.assert_allclose(w, expect, rtol=0, atol=2e-16 * 4)


@pytest.mark.parametrize("case", [c for c in GOLDEN["cases"] if c["kernel"] in ("IB_3", "PIECEWISE_CUBIC")],
                         ids=lambda c: f"{c['kernel']}@{c['X_o_dx']}")
def test_pointwise_kernels_known_answer(oracle, case):
    """IB_3 / PIECEWISE_CUBIC via a 1-cell-thick 2-D interpolation of unit vectors."""
    k = case["kernel"]
    x = float(case["X_o_dx"])
    expect = [float(Decimal(v)) for v in case["w"]]
    # 2-D grid wide enough in x; the y coordinate sits at a cell centre so the
    # y weights are (0, 1, 0) for IB_3 and (phi(-1), phi(0), phi(1), ...) for pw-cubic
    lo, hi, g = [-20, 0], [20, 0], [4, 4]
    shape = oracle.ghost_shape(lo, hi, g)
    X = np.array([[x, 0.5]])
    got = []
    for j in range(case["ic_lower"], case["ic_lower"] + len(expect)):
        u = np.zeros(shape)
        u[0, :, j - (lo[0] - g[0])] = 1.0  # whole y column at x-index j
        V = np.zeros(1)
        oracle.interp(k, [1.0, 1.0], [float(lo[0]), 0.0], lo, hi, g, u, [0], np.zeros((1, 2)), X, V)
        got.append(V[0])
    # the y-sum of weights is 1 (partition of unity) up to rounding
    np.testing.assert_allclose(got, expect, rtol=0, atol=4e-15)


def _indicator_interp(oracle, kernel, x, j, axis=0):
    """V at X_o_dx = x (2-D, dx = 1, x_lower = 0, y at a cell centre) of the field
    that is 1 on the whole grid column x-index j: the x weight of point j."""
    # x_lower = 0 and ilower = 0, so X_o_dx = x exactly (NINT is not shift-invariant:
    # NINT(-0.5) = -1 puts X = 0 in cell -1 for the low-order kernels)
    lo, hi, g = [0, 0], [20, 0], [4, 4]
    u = np.zeros(oracle.ghost_shape(lo, hi, g))
    u[0, :, j - (lo[0] - g[0])] = 1.0
    V = np.zeros(1)
    oracle.interp(kernel, [1.0, 1.0], [0.0, 0.0], lo, hi, g, u, [0], np.zeros((1, 2)),
                  np.array([[x, 0.5]]), V, axis=axis)
    return V[0]


LOW = [c for c in GOLDEN["cases"] if c["kernel"] in ("PIECEWISE_LINEAR", "DISCONTINUOUS_LINEAR", "PIECEWISE_CONSTANT")]


@pytest.mark.parametrize("case", LOW, ids=lambda c: f"{c['kernel']}@{c['X_o_dx']}{'' if c.get('axis_dim', True) else '-offaxis'}")
def test_low_order_kernels_known_answer(oracle, case):
    """PIECEWISE_LINEAR / DISCONTINUOUS_LINEAR / PIECEWISE_CONSTANT: the weight of
    every stencil point, and zero just outside the stencil (its placement)."""
    x = float(case["X_o_dx"])
    axis = 0 if case.get("axis_dim", True) else 1  # DISCONTINUOUS_LINEAR: x is the axis dim or not
    expect = [float(Decimal(v)) for v in case["w"]]
    icl = case["ic_lower"]
    got = [_indicator_interp(oracle, case["kernel"], x, icl + k, axis) for k in range(len(expect))]
    np.testing.assert_allclose(got, expect, rtol=0, atol=4e-15)
    for j in (icl - 1, icl + len(expect)):
        assert _indicator_interp(oracle, case["kernel"], x, j, axis) == 0.0


def test_nint_half_away_from_zero(oracle):
    # NINT(2.5) = 3, NINT(-2.5) = -3 (F7); IB_4 ic_lower = NINT(x) - 2
    assert oracle.weights_1d("IB_4", 2.5)[0] == 1
    assert oracle.weights_1d("IB_4", -2.5)[0] == -5
    assert oracle.weights_1d("IB_4", 2.4999999999999996)[0] == 0


def test_lagrangian_floor_quirk(oracle):
    # int(x) - (x<0): -2.0 -> -3 (a6)
    L = oracle.lib()
    assert L.ora_lagrangian_floor(-2.0) == -3
    assert L.ora_lagrangian_floor(-1.5) == -2
    assert L.ora_lagrangian_floor(1.5) == 1
    assert L.ora_lagrangian_floor(0.0) == 0


def _moments(oracle, kernel, x):
    icl, w = oracle.weights_1d(kernel, x)
    d = x - (np.arange(icl, icl + w.size) + 0.5)
    return w, d


@pytest.mark.parametrize("kernel", ["IB_4", "IB_4_W8", "IB_6", "BSPLINE_4"])
def test_closed_form_moments(oracle, kernel):
    rng = np.random.default_rng(7)
    for x in np.concatenate([rng.uniform(-50, 50, 200), [0.5, 1.0, 2.5, -2.5]]):
        w, d = _moments(oracle, kernel, x)
        assert abs(w.sum() - 1.0) < 4e-15
        assert abs((w * d).sum()) < 4e-14
        if kernel == "IB_4":
            assert abs((w * w).sum() - 3.0 / 8.0) < 4e-15  # Peskin's sum-of-squares condition
            assert abs(w[0::2].sum() - 0.5) < 4e-15  # even-odd condition
        if kernel == "IB_6":
            K = (59.0 / 60.0) * (1.0 - np.sqrt(1.0 - 3220.0 / 3481.0))
            assert abs(w[0::2].sum() - 0.5) < 4e-15
            assert abs((w * d * d).sum() - K) < 4e-14  # second moment = K
            assert abs((w * d ** 3).sum()) < 4e-13
        assert (w >= -1e-15).all() or kernel == "IB_6"


# ---------------------------------------------------------------------------
# whole-call identities
# ---------------------------------------------------------------------------
def _grid(ndim, N, g):
    lo = [0] * ndim
    hi = [N - 1] * ndim
    return lo, hi, [g] * ndim


@pytest.mark.parametrize("kernel", ALL)
@pytest.mark.parametrize("ndim", [2, 3])
def test_interp_constant_and_linear(oracle, kernel, ndim):
    N = 12
    g = oracle.min_ghost_width(kernel) + 1
    lo, hi, gw = _grid(ndim, N, g)
    dx = [1.0 / N] * ndim
    xlo = [0.0] * ndim
    rng = np.random.default_rng(1)
    M = 50
    X = rng.uniform(0.3, 0.7, (M, ndim))
    idx = np.arange(M, dtype=np.int32)
    xs = np.zeros((M, ndim))
    shape = oracle.ghost_shape(lo, hi, gw)
    V = np.zeros(M)
    oracle.interp(kernel, dx, xlo, lo, hi, gw, np.full(shape, 2.5), idx, xs, X, V, axis=0)
    np.testing.assert_allclose(V, 2.5, rtol=0, atol=1e-13)
    if kernel in SMOOTH:
        # u = cell-centre x coordinate -> interp reproduces X[:, 0]
        n0 = shape[-1]
        xc = (np.arange(n0) + (lo[0] - g) + 0.5) / N
        u = np.broadcast_to(xc, shape).copy()
        oracle.interp(kernel, dx, xlo, lo, hi, gw, u, idx, xs, X, V)
        np.testing.assert_allclose(V, X[:, 0], rtol=0, atol=1e-13)


@pytest.mark.parametrize("kernel", ALL)
@pytest.mark.parametrize("ndim", [2, 3])
def test_spread_conservation_and_adjointness(oracle, kernel, ndim):
    N = 12
    g = oracle.min_ghost_width(kernel) + 1
    lo, hi, gw = _grid(ndim, N, g)
    dx = [1.0 / N] * ndim
    h = np.prod(dx)
    xlo = [0.0] * ndim
    rng = np.random.default_rng(2)
    M = 40
    X = rng.uniform(0.3, 0.7, (M, ndim))
    idx = np.arange(M, dtype=np.int32)
    xs = np.zeros((M, ndim))
    shape = oracle.ghost_shape(lo, hi, gw)
    F = rng.standard_normal(M)
    f = np.zeros(shape)
    oracle.spread(kernel, dx, xlo, lo, hi, gw, f, idx, xs, X, F)
    assert abs(f.sum() * h - F.sum()) < 1e-12 * max(1.0, np.abs(F).sum())
    u = rng.standard_normal(shape)
    U = np.zeros(M)
    oracle.interp(kernel, dx, xlo, lo, hi, gw, u, idx, xs, X, U)
    lhs = (f * u).sum() * h
    rhs = (F * U).sum()
    assert abs(lhs - rhs) < 1e-12 * max(1.0, abs(rhs), np.abs(F).sum())


@pytest.mark.parametrize("kernel", ["IB_4", "IB_6", "PIECEWISE_LINEAR", "PIECEWISE_CUBIC", "IB_3"])
def test_clipping_at_ghost_box_edge(oracle, kernel):
    """Markers near/outside the ghost box: stencils are clipped, never read/written out of range."""
    N, g = 8, oracle.min_ghost_width(kernel)
    lo, hi, gw = _grid(3, N, g)
    dx = [1.0 / N] * 3
    shape = oracle.ghost_shape(lo, hi, gw)
    guard = 7
    buf = np.full(np.prod(shape) + 2 * guard, 123.0)
    u = buf[guard:-guard].reshape(shape)
    u[...] = 0.0
    X = np.array([[-(g + 0.9) / N, 0.5, 0.5], [(N + g + 0.9) / N, 0.5, 0.5], [-0.01, -0.01, 1.01], [0.5, 0.5, 0.5]])
    F = np.ones(4)
    oracle.spread(kernel, dx, [0, 0, 0], lo, hi, gw, u, np.arange(4), np.zeros((4, 3)), X, F)
    assert (buf[:guard] == 123.0).all() and (buf[-guard:] == 123.0).all()
    V = np.full(4, np.nan)
    oracle.interp(kernel, dx, [0, 0, 0], lo, hi, gw, u, np.arange(4), np.zeros((4, 3)), X, V)
    assert np.isfinite(V).all()


def test_side_wrapper_periodic_images_match_unwrapped(oracle):
    """Spreading the periodic index list on a ghosted periodic patch gives the
    same interior values as spreading the unwrapped markers on a bigger grid."""
    N, g, kernel = 10, 3, "IB_4"
    lo, hi = [0, 0, 0], [N - 1] * 3
    dx = [1.0 / N] * 3
    rng = np.random.default_rng(3)
    M = 30
    X = rng.uniform(0, 1, (M, 3))
    Fm = rng.standard_normal((M, 3))
    idx, xs, _ = oracle.periodic_index_list(X, [0, 0, 0], [1, 1, 1], dx, lo, hi, g)
    assert idx.size > M  # some images
    f = [np.zeros(oracle.ghost_shape(*oracle.side_box(lo, hi, a), [g] * 3)) for a in range(3)]
    oracle.side_spread(kernel, dx, [0, 0, 0], lo, hi, [g] * 3, f, idx, xs, X, Fm)
    # brute force: sum the 27 images on an unghosted periodic grid
    ref = [np.zeros((N, N, N)) for _ in range(3)]
    import itertools
    for a in range(3):
        big_lo, big_hi = [-N] * 3, [2 * N - 1] * 3
        fb = np.zeros(oracle.ghost_shape(*oracle.side_box(big_lo, big_hi, a), [g] * 3))
        for sh in itertools.product((-1, 0, 1), repeat=3):
            Xs = X + np.array(sh)[None, :]
            xl = [0.0, 0.0, 0.0]
            xl[a] -= 0.5 * dx[a]
            blo, bhi = oracle.side_box(big_lo, big_hi, a)
            # note: the big patch has x_lower at -1 (cell -N)
            xl = [v - 1.0 for v in xl]
            oracle.spread(kernel, dx, xl, blo, bhi, [g] * 3, fb, np.arange(M), np.zeros((M, 3)), Xs, Fm[:, a].copy())
        off = g + N
        ref[a] = fb[0, off:off + N, off:off + N, off:off + N]
        got = f[a][0, g:g + N, g:g + N, g:g + N]
        np.testing.assert_allclose(got, ref[a], rtol=0, atol=1e-9 * np.abs(ref[a]).max())


def test_oracle_side_ib4_known_answer_3d(oracle):
    """The oracle's 3-D side-centred IB_4 interp and spread against the 50-digit decimal
    known answers of tests/golden/kat3d_side_ib4.json (tests/golden/make_kat3d.py, from
    the Fortran text and LEInteractor's side frame shifts; clipped stencils, periodic
    images, a repeated list entry)."""
    import json
    from pathlib import Path
    k = json.loads((Path(__file__).parent / "golden" / "kat3d_side_ib4.json").read_text())
    X = np.array(k["X"])
    idx = np.array(k["indices"], dtype=np.int32)
    xs = np.array(k["Xshift"])
    u = [np.array(a) for a in k["u"]]
    gcw = [k["gcw"]] * 3
    Q = np.zeros_like(X)
    oracle.side_interp("IB_4", k["dx"], k["x_lower"], k["ilower"], k["iupper"], gcw, [a.copy() for a in u], idx, xs,
                       X, Q)
    Qe = np.array(k["Q"])
    assert np.abs(Q - Qe).max() <= 1e-14 * np.abs(Qe).max()
    uo = [a.copy() for a in u]
    oracle.side_spread("IB_4", k["dx"], k["x_lower"], k["ilower"], k["iupper"], gcw, uo, idx, xs, X, np.array(k["F"]))
    for a in range(3):
        fe = np.array(k["f"][a])
        assert np.abs(uo[a] - fe).max() <= 1e-13 * np.abs(fe).max()


# ---------------------------------------------------------------------------- every kernel
def _kat_cases():
    import json
    from pathlib import Path
    return json.loads((Path(__file__).parent / "golden" / "kat_kernels.json").read_text())["cases"]


KAT_CASES = _kat_cases()


def kat_arrays(case):
    """The case's component arrays (numpy, C order) from the u formula of make_kat.py, and
    each array's (x_lower frame, box lo, box hi, DISCONTINUOUS_LINEAR axis)."""
    nd, g, dep = case["ndim"], case["gcw"], case["depth"]
    lo, hi, dx, xl = case["ilower"], case["iupper"], case["dx"], case["x_lower"]
    cent = case["centering"]
    frames = []
    if cent == "cell":
        frames.append((list(xl), list(lo), list(hi), case["axis"]))
    elif cent == "node":
        frames.append(([xl[d] - 0.5 * dx[d] for d in range(nd)], list(lo), [h + 1 for h in hi], case["axis"]))
    else:
        for a in range(nd):
            if cent == "side":
                x2 = [xl[d] - (0.5 * dx[d] if d == a else 0.0) for d in range(nd)]
                h2 = [hi[d] + (1 if d == a else 0) for d in range(nd)]
            else:
                x2 = [xl[d] - (0.5 * dx[d] if d != a else 0.0) for d in range(nd)]
                h2 = [hi[d] + (1 if d != a else 0) for d in range(nd)]
            frames.append((x2, list(lo), h2, a))
    arrays = []
    for c, (_, blo, bhi, _) in enumerate(frames):
        shape = [bhi[d] - blo[d] + 1 + 2 * g for d in range(nd)][::-1]
        if cent in ("cell", "node"):
            shape = [dep] + shape
        n = int(np.prod(shape))
        i = np.arange(n, dtype=np.int64)
        arrays.append((((i * 7919 + c * 104729 + case["useed"]) % 33 - 16) / 8.0).reshape(shape))
    return arrays, frames


def kat_expected_f(case, arrays):
    out = []
    for c, a in enumerate(arrays):
        e = a.copy().reshape(-1)
        for flat, v in case["f"][c]:
            e[flat] = v
        out.append(e.reshape(a.shape))
    return out


def kat_id(case):
    return f'{case["kernel"]}-{case["ndim"]}d-{case["centering"]}'


@pytest.mark.parametrize("case", KAT_CASES, ids=kat_id)
def test_oracle_known_answers_every_kernel(oracle, case):
    """The oracle (le_oracle.c) against the 50-digit decimal evaluations of the Fortran text
    (tests/golden/make_kat.py) for every reference kernel function, 2-D and 3-D, on cell,
    node, side and edge data: clipped stencils, NINT ties, lagrangian_floor at negative
    integers, PIECEWISE_CUBIC's unshifted side test, periodic images, a repeated entry.
    Interp within 1e-14, spread within 1e-13 (relative to the largest magnitude)."""
    k = case
    nd, g, dep = k["ndim"], k["gcw"], k["depth"]
    X = np.array(k["X"])
    idx = np.array(k["indices"], dtype=np.int32)
    xs = np.array(k["Xshift"])
    F = np.array(k["F"])
    Qe = np.array(k["Q"], dtype=np.float64)
    arrays, frames = kat_arrays(k)
    gcw = [g] * nd
    per_axis = k["centering"] in ("side", "edge")
    Q = np.zeros_like(Qe)
    fo = [a.copy() for a in arrays]
    for c, (xl, lo, hi, ax) in enumerate(frames):
        depth = 1 if per_axis else dep
        V = np.zeros((X.shape[0], depth))
        oracle.interp(k["kernel"], k["dx"], xl, lo, hi, gcw, arrays[c].copy(), idx, xs, X, V, depth=depth, axis=ax)
        if per_axis:
            Q[:, c] = V[:, 0]
        else:
            Q[:, :] = V
        Fv = np.ascontiguousarray(F[:, c:c + 1] if per_axis else F[:, :dep])
        oracle.spread(k["kernel"], k["dx"], xl, lo, hi, gcw, fo[c], idx, xs, X, Fv, depth=depth, axis=ax)
    assert np.abs(Q - Qe).max() <= 1e-14 * max(np.abs(Qe).max(), 1.0), kat_id(k)
    for c, fe in enumerate(kat_expected_f(k, arrays)):
        assert np.abs(fo[c] - fe).max() <= 1e-13 * np.abs(fe).max(), (kat_id(k), c)
