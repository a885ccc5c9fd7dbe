"""GPU: ibtk_le_fill_interp_update -- the periodic fill, the interp and IBMethod::eulerStep's
position update (IBMethod.cpp:619-655: X_new = dt U + X) in one sweep -- against the three
calls it replaces (fill_interp, then position_update("euler", dt, X, Q)): Q and X_new bit for
bit, in place and out of place.  Cases: closed-form, piecewise-linear and piecewise-cubic
kernels (the last reads X itself: out of place only); an index list with repeated entries
(a marker's row written once); markers binned outside the patch (Q = 0, X unchanged); the
argument checks (shifted lists, in-place piecewise cubic, Q_depth)."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def le():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from ibamr_amd import le as _le
    return _le


def _err():
    from ibamr_amd._lib import IBTKLEError
    return IBTKLEError


def _field(geom, rng):
    u = geom.alloc("side")
    for a in u:
        a.copy_(torch.from_numpy(rng.uniform(-1, 1, tuple(a.shape))))
    return u


def _reference(le, ctx, m, kernel, geom, u, X, dt, periodic):
    Q = torch.zeros_like(X)
    le.fill_interp(ctx, m, kernel, "side", geom, u, Q, X, periodic=periodic)
    Xn = torch.empty_like(X)
    le.position_update(ctx, "euler", dt, X, Q, out=Xn)
    ctx.synchronize()
    return Q, Xn


@pytest.mark.parametrize("kernel", ["IB_4", "IB_6", "PIECEWISE_LINEAR", "PIECEWISE_CUBIC"])
def test_fused_update_equals_interp_then_euler(le, kernel):
    N = (48, 40, 56)
    g = le._lib.load().ibtk_le_min_ghost_width(le.kernel_id(kernel))
    geom = le.Geometry.periodic_unit(list(N), g)
    rng = np.random.default_rng(21)
    M = 30000
    X = torch.from_numpy(rng.uniform(0.0, 1.0, (M, 3))).cuda()
    u = _field(geom, rng)
    ctx = le.Context(0)
    m = le.Markers(ctx).bin(geom, kernel, X)
    dt = 0.37 / N[0]
    Q0, X0 = _reference(le, ctx, m, kernel, geom, u, X, dt, [1, 1, 1])
    Q1 = torch.zeros_like(X)
    X1 = torch.full_like(X, float("nan"))
    le.fill_interp_update(ctx, m, kernel, "side", geom, u, Q1, X, dt, X_out=X1, periodic=[1, 1, 1])
    ctx.synchronize()
    assert torch.equal(Q1, Q0)
    assert torch.equal(X1, X0)
    if kernel != "PIECEWISE_CUBIC":
        X2 = X.clone()
        Q2 = torch.zeros_like(X)
        le.fill_interp_update(ctx, m, kernel, "side", geom, u, Q2, X2, dt, periodic=[1, 1, 1])  # in place
        ctx.synchronize()
        assert torch.equal(Q2, Q0)
        assert torch.equal(X2, X0)
    else:
        with pytest.raises(_err()):
            le.fill_interp_update(ctx, m, kernel, "side", geom, u, Q1, X, dt, periodic=[1, 1, 1])


def test_fused_update_repeated_entries_and_outside_markers(le):
    """A patch covering part of the domain (no periodic dims): markers beyond its ghost box
    are binned outside (Q = 0, X_new = X); an index list naming markers twice writes each
    row once, and rows the list does not name are left alone."""
    kernel = "IB_4"
    geom = le.Geometry((8, 4, 0), (39, 27, 31), 3, [1.0 / 64] * 3, [8 / 64, 4 / 64, 0.0])
    rng = np.random.default_rng(4)
    M = 20000
    X = torch.from_numpy(rng.uniform(0.0, 0.75, (M, 3))).cuda()
    u = _field(geom, rng)
    ctx = le.Context(0)
    idx = torch.from_numpy(np.concatenate([np.arange(0, M, 2), rng.integers(0, M, 3000)]).astype(np.int32)).cuda()
    m = le.Markers(ctx).bin(geom, kernel, X, idx)
    dt = -0.01
    Q0, X0 = _reference(le, ctx, m, kernel, geom, u, X, dt, [0, 0, 0])
    Q1 = torch.zeros_like(X)
    X1 = torch.full_like(X, 7.0)
    le.fill_interp_update(ctx, m, kernel, "side", geom, u, Q1, X, dt, X_out=X1, periodic=[0, 0, 0])
    ctx.synchronize()
    named = torch.zeros(M, dtype=torch.bool, device="cuda")
    named[idx.long()] = True
    assert torch.equal(Q1[named], Q0[named])
    assert torch.equal(X1[named], X0[named])
    assert torch.all(X1[~named] == 7.0)
    assert (Q1[named] == 0).all(dim=1).any()  # some named markers lie outside every stencil's reach


def test_fused_update_argument_checks(le):
    geom = le.Geometry.periodic_unit([32, 32, 32], 3)
    rng = np.random.default_rng(6)
    M = 1000
    X = torch.from_numpy(rng.uniform(0.0, 1.0, (M, 3))).cuda()
    u = _field(geom, rng)
    ctx = le.Context(0)
    idx = torch.arange(M, dtype=torch.int32, device="cuda")
    shift = torch.zeros((M, 3), dtype=torch.float64, device="cuda")
    m = le.Markers(ctx).bin(geom, "IB_4", X, idx, shift)
    Q = torch.zeros_like(X)
    with pytest.raises(_err()):  # a list with periodic shifts
        le.fill_interp_update(ctx, m, "IB_4", "side", geom, u, Q, X, 0.1, X_out=X.clone())
    m2 = le.Markers(ctx).bin(geom, "IB_4", X)
    c = geom.alloc("cell")
    with pytest.raises(_err()):  # depth-1 cell data: one component, not NDIM
        le.fill_interp_update(ctx, m2, "IB_4", "cell", geom, c, torch.zeros((M, 1), dtype=torch.float64,
                                                                             device="cuda"), X, 0.1,
                              X_out=X.clone(), Q_depth=1)
