"""GPU: marker position update (ibtk_le_position_update).

IBMethod::eulerStep / midpointStep / trapezoidalStep (IBMethod.cpp:619-681) are
PETSc VecWAXPY (w = a x + y) and VecAXPY (y = a x + y): a rounded multiply then a
rounded add per element.  numpy computes the same two roundings, so the device
result must match bit for bit.
"""
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


@pytest.fixture(scope="module")
def ctx(le):
    return le.Context(0)


def _ref(scheme, dt, X, U0, U1):
    if scheme == "trapezoidal":
        h = 0.5 * dt
        return (h * U0 + X) + h * U1
    return dt * U0 + X


@pytest.mark.parametrize("scheme", ["euler", "midpoint", "trapezoidal"])
@pytest.mark.parametrize("M", [1, 7, 4096, 100_003])
def test_update_bitwise(le, ctx, scheme, M):
    rng = np.random.default_rng(M)
    X = rng.random((M, 3)) * 10 - 5
    U0 = rng.standard_normal((M, 3))
    U1 = rng.standard_normal((M, 3))
    dt = 1.0 / 3.0e3
    Xd, U0d, U1d = (torch.from_numpy(a).cuda() for a in (X, U0, U1))
    out = le.position_update(ctx, scheme, dt, Xd, U0d, U1d)
    ctx.synchronize()
    assert np.array_equal(out.cpu().numpy(), _ref(scheme, dt, X, U0, U1))


def test_update_in_place_and_unaligned(le, ctx):
    """In-place (X_new = X_cur) and an odd, 8-byte-offset view take the scalar path."""
    rng = np.random.default_rng(1)
    n = 3 * 1001
    base = torch.from_numpy(rng.random(n + 1)).cuda()
    X = base[1:]                      # 8-byte offset from a 16-byte-aligned allocation
    U = torch.from_numpy(rng.random(n)).cuda()
    ref = _ref("euler", 0.25, X.cpu().numpy(), U.cpu().numpy(), None)
    le.position_update(ctx, "euler", 0.25, X, U, out=X)
    ctx.synchronize()
    assert np.array_equal(X.cpu().numpy(), ref)


def test_update_errors(le, ctx):
    X = torch.zeros((4, 3), dtype=torch.float64, device="cuda:0")
    with pytest.raises(ValueError):
        le.position_update(ctx, "trapezoidal", 0.1, X, X)
    with pytest.raises(ValueError):
        le.position_update(ctx, "rk4", 0.1, X, X)
    lib = le._lib.load()
    assert lib.ibtk_le_position_update(ctx.h, 7, 12, 0.1, None, None, None, None) != 0
    assert lib.ibtk_le_position_update(ctx.h, 0, 0, 0.1, None, None, None, None) == 0


def test_update_then_rebin_interp(le, ctx, oracle):
    """One explicit step of the coupling loop on the device: interp U at X, X += dt U,
    re-bin, interp again; the second interp matches the oracle at the moved positions."""
    from ibamr_amd.le import Geometry
    kernel = "IB_4"
    geom = Geometry.periodic_unit([16, 16, 16], oracle.min_ghost_width(kernel))
    g = torch.Generator(device="cuda:0").manual_seed(9)
    M = 2000
    X = 0.2 + 0.6 * torch.rand((M, 3), dtype=torch.float64, device="cuda:0", generator=g)
    u = geom.alloc("side")
    for a in u:
        a.uniform_(-1.0, 1.0, generator=g)
    le.fill_periodic_ghosts(ctx, geom, "side", u)
    U = torch.zeros_like(X)
    m = le.Markers(ctx).bin(geom, kernel, X)
    le.interp(ctx, m, kernel, "side", geom, u, U, X)
    X1 = le.position_update(ctx, "euler", 0.01, X, U)
    m.bin(geom, kernel, X1)
    U1 = torch.zeros_like(X)
    le.interp(ctx, m, kernel, "side", geom, u, U1, X1)
    ctx.synchronize()
    Xn = X1.cpu().numpy()
    assert np.array_equal(Xn, 0.01 * U.cpu().numpy() + X.cpu().numpy())
    Uo = np.zeros((M, 3))
    u0 = [a.cpu().numpy() for a in u]
    oracle.side_interp(kernel, geom.dx, geom.x_lower, geom.ilower, geom.iupper, geom.gcw, u0,
                       np.arange(M, dtype=np.int32), np.zeros((M, 3)), Xn, Uo)
    scale = np.abs(Uo).max()
    assert np.abs(U1.cpu().numpy() - Uo).max() / scale <= 1e-13


def test_moving_step_has_no_host_sync(le, ctx):
    """One explicit coupling step on one GPU -- ghost fill, interp, X += dt U, re-bin,
    zero ghosts, spread, fold (bench.py --move at N = 1) -- issues no host
    synchronisation: torch's sync debug mode set to "error" stays silent (the library
    calls themselves only enqueue work on the context stream), and the results match
    the same step run with the mode off."""
    from ibamr_amd.le import Geometry
    N = 48
    geom = Geometry.periodic_unit([N, N, N], 3)
    g = torch.Generator(device="cuda:0").manual_seed(11)
    M = 20000
    X0 = torch.rand((M, 3), dtype=torch.float64, device="cuda", generator=g)
    F = torch.rand((M, 3), dtype=torch.float64, device="cuda", generator=g) - 0.5
    u = geom.alloc("side")
    for a in u:
        a.uniform_(-1, 1, generator=g)
    dt = 0.05 / N

    def step(X, U, f, bins):
        le.fill_periodic_ghosts(ctx, geom, "side", u)
        le.interp(ctx, bins, "IB_4", "side", geom, u, U, X)
        le.position_update(ctx, "euler", dt, X, U, out=X)
        bins.bin(geom, "IB_4", X)
        le.zero_ghosts(ctx, geom, "side", f)
        le.spread(ctx, bins, "IB_4", "side", geom, f, F, X)
        le.fold_periodic_ghosts(ctx, geom, "side", f)

    outs = []
    for mode in ("error", None):
        X = X0.clone()
        U = torch.zeros_like(X)
        f = geom.alloc("side")
        bins = le.Markers(ctx).bin(geom, "IB_4", X)
        step(X, U, f, bins)  # first call: the library's buffers are allocated here
        ctx.synchronize()
        if mode:
            torch.cuda.set_sync_debug_mode(mode)
        try:
            step(X, U, f, bins)
        finally:
            torch.cuda.set_sync_debug_mode(0)
        ctx.synchronize()
        outs.append((X.clone(), U.clone(), [a.clone() for a in f]))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    assert all(torch.equal(a, b) for a, b in zip(outs[0][2], outs[1][2]))
