"""GPU parity: the HIP path (through the C-ABI) against the oracle, on the GPU.

Bar (BASELINE.json north_star): interp fp64 relative error <= 1e-13, spread
<= 1e-12 with a deterministic order, bit-stable run to run.  The oracle is fed
the exact list order the GPU sums in (ibtk_le_markers_order), so the kernels
are expected to agree with it bit for bit (both built with -ffp-contract=off);
the tests assert the stated tolerances and report bitwise agreement separately.
"""
import zlib

import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

ALL = ["PIECEWISE_CONSTANT", "DISCONTINUOUS_LINEAR", "PIECEWISE_LINEAR", "PIECEWISE_CUBIC", "IB_3", "IB_4",
       "IB_4_W8", "IB_6", "BSPLINE_4"]
INTERP_TOL = 1e-13
SPREAD_TOL = 1e-12


@pytest.fixture(scope="module")
def le():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from ibamr_amd import le as _le
    return _le


@pytest.fixture(scope="module")
def ctx(le):
    return le.Context(0)


def rel_err(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    scale = max(np.abs(b).max(), 1e-300) if b.size else 1.0
    return float(np.abs(a - b).max() / scale) if a.size else 0.0


def make_case(kernel, ndim, centering, seed, M=300, extra_ghost=0, shifts=True, subset=True):
    rng = np.random.default_rng(seed)
    N = 13 if ndim == 3 else 29
    ilower = [3, -2, 5][:ndim]
    iupper = [ilower[d] + N - 1 + d for d in range(ndim)]
    from oracle.oracle import min_ghost_width
    g = min_ghost_width(kernel) + extra_ghost
    dx = [0.1, 0.07, 0.05][:ndim]
    xlo = [-0.3, 0.2, 1.0][:ndim]
    from ibamr_amd.le import Geometry
    geom = Geometry(ilower, iupper, g, dx, xlo)
    L = np.array([(iupper[d] - ilower[d] + 1) * dx[d] for d in range(ndim)])
    # markers: mostly inside, some within the ghost layer, a few far outside
    X = xlo + rng.uniform(-0.1, 1.1, (M, ndim)) * L
    X[:5] = xlo + rng.uniform(-2.0, 3.0, (5, ndim)) * L
    # exact cell faces / centres (NINT ties)
    X[5:10, 0] = xlo[0] + (np.arange(5) + 2) * dx[0] * 0.5
    if subset:
        idx = rng.permutation(M)[: M - 37].astype(np.int32)
    else:
        idx = np.arange(M, dtype=np.int32)
    n = idx.size
    xs = np.zeros((n, ndim))
    if shifts:
        pick = rng.random(n) < 0.2
        xs[pick] = rng.integers(-1, 2, (pick.sum(), ndim)) * L
    depth = {"side": 1, "edge": 1, "cell": 2, "node": 1}[centering]
    return geom, X, idx, xs, depth


def oracle_call(ora, op, kernel, centering, geom, u_list, idx, xs, X, Q, depth):
    lo, hi = list(geom.ilower), list(geom.iupper)
    gcw = list(geom.gcw)
    dx, xl = list(geom.dx), list(geom.x_lower)
    nd = geom.ndim
    if centering == "side":
        f = ora.side_interp if op == "interp" else ora.side_spread
        return f(kernel, dx, xl, lo, hi, gcw, u_list, idx, xs, X, Q)
    if centering == "edge":
        for axis in range(nd):
            xla = [xl[d] - (0.5 * dx[d] if d != axis else 0.0) for d in range(nd)]
            hia = [hi[d] + (1 if d != axis else 0) for d in range(nd)]
            if op == "interp":
                Qa = np.zeros(int(idx.max()) + 1)
                ora.interp(kernel, dx, xla, lo, hia, gcw, u_list[axis], idx, xs, X, Qa, depth=1, axis=axis)
                Q.reshape(-1, nd)[idx, axis] = Qa[idx]
            else:
                Qa = np.zeros(int(idx.max()) + 1)
                Qa[idx] = Q.reshape(-1, nd)[idx, axis]
                ora.spread(kernel, dx, xla, lo, hia, gcw, u_list[axis], idx, xs, X, Qa, depth=1, axis=axis)
        return
    if centering == "cell":
        f = ora.cell_interp if op == "interp" else ora.cell_spread
    else:
        f = ora.node_interp if op == "interp" else ora.node_spread
    return f(kernel, dx, xl, lo, hi, gcw, u_list[0], idx, xs, X, Q, depth)


CASES = [(k, nd, c) for k in ALL for nd in (2, 3) for c in ("side", "cell", "node", "edge")
         if not (c == "edge" and nd == 2)]


@pytest.mark.parametrize("kernel,ndim,centering", CASES, ids=lambda v: str(v))
def test_interp_matches_oracle(le, ctx, oracle, kernel, ndim, centering):
    geom, X, idx, xs, depth = make_case(kernel, ndim, centering, seed=zlib.crc32(f'{kernel}{ndim}{centering}'.encode()))
    rng = np.random.default_rng(11)
    dev = "cuda:0"
    q = geom.alloc(centering, depth)
    for a in q:
        a.copy_(torch.from_numpy(rng.uniform(-1, 1, tuple(a.shape))))
    Xd = torch.from_numpy(X).to(dev)
    idd = torch.from_numpy(idx).to(dev)
    xsd = torch.from_numpy(xs).to(dev)
    Qdepth = ndim if centering in ("side", "edge") else depth
    Q = torch.full((X.shape[0], Qdepth), np.nan, dtype=torch.float64, device=dev)
    m = le.Markers(ctx).bin(geom, kernel, Xd, idd, xsd)
    le.interp(ctx, m, kernel, centering, geom, q, Q, Xd, q_depth=depth)
    ctx.synchronize()
    Qg = Q.cpu().numpy()
    Qo = np.full_like(Qg, np.nan)
    u_np = [a.cpu().numpy().copy() for a in q]
    oracle_call(oracle, "interp", kernel, centering, geom, u_np, idx, xs, X, Qo, depth)
    listed = np.zeros(X.shape[0], bool)
    listed[idx] = True
    assert np.isnan(Qg[~listed]).all(), "unlisted markers must be untouched"
    err = rel_err(Qg[listed], Qo[listed])
    assert err <= INTERP_TOL, f"interp rel err {err:.3e}"
    bitwise = np.array_equal(Qg[listed], Qo[listed])
    print(f"{kernel} {ndim}d {centering}: interp rel err {err:.2e} bitwise={bitwise}")


@pytest.mark.parametrize("kernel,ndim,centering", CASES, ids=lambda v: str(v))
def test_spread_matches_oracle_in_canonical_order(le, ctx, oracle, kernel, ndim, centering):
    geom, X, idx, xs, depth = make_case(kernel, ndim, centering, seed=1 + zlib.crc32(f'{kernel}{ndim}{centering}'.encode()))
    rng = np.random.default_rng(12)
    dev = "cuda:0"
    q = geom.alloc(centering, depth)
    for a in q:
        a.copy_(torch.from_numpy(rng.uniform(-1, 1, tuple(a.shape))))
    u0 = [a.cpu().numpy().copy() for a in q]
    Qdepth = ndim if centering in ("side", "edge") else depth
    F = rng.uniform(-1, 1, (X.shape[0], Qdepth))
    Xd, Fd = torch.from_numpy(X).to(dev), torch.from_numpy(F).to(dev)
    idd, xsd = torch.from_numpy(idx).to(dev), torch.from_numpy(xs).to(dev)
    m = le.Markers(ctx).bin(geom, kernel, Xd, idd, xsd)
    le.spread(ctx, m, kernel, centering, geom, q, Fd, Xd, q_depth=depth)
    ctx.synchronize()
    order = m.order().cpu().numpy()
    assert sorted(order.tolist()) == list(range(idx.size))
    ug = [a.cpu().numpy() for a in q]
    uo = [a.copy() for a in u0]
    oracle_call(oracle, "spread", kernel, centering, geom, uo, idx[order], xs[order], X, F.copy(), depth)
    uc = [a.copy() for a in u0]  # the caller's list order (the reference's summation order)
    oracle_call(oracle, "spread", kernel, centering, geom, uc, idx, xs, X, F.copy(), depth)
    for a in range(len(ug)):
        err = rel_err(ug[a], uo[a])
        assert err <= SPREAD_TOL, f"spread comp {a} rel err {err:.3e}"
        err = rel_err(ug[a], uc[a])
        assert err <= SPREAD_TOL, f"spread comp {a} rel err {err:.3e} against the caller's order"
    bitwise = all(np.array_equal(ug[a], uo[a]) for a in range(len(ug)))
    print(f"{kernel} {ndim}d {centering}: spread bitwise={bitwise}")


@pytest.mark.parametrize("kernel", ["IB_4", "IB_6", "PIECEWISE_LINEAR", "BSPLINE_4"])
def test_bitwise_against_oracle_ib_side(le, ctx, oracle, kernel):
    """The headline path (3-D side-centred): interpolation matches the oracle
    bit for bit; spreading sums each grid point's contributions in the kernel's
    fixed (phase, class, stencil point, lane) order, i.e. the Fortran's
    sequential sum reassociated, so it is held to the stated 1e-12."""
    geom, X, idx, xs, depth = make_case(kernel, 3, "side", seed=5, M=2000)
    rng = np.random.default_rng(3)
    dev = "cuda:0"
    q = geom.alloc("side")
    for a in q:
        a.copy_(torch.from_numpy(rng.uniform(-1, 1, tuple(a.shape))))
    u0 = [a.cpu().numpy().copy() for a in q]
    F = rng.uniform(-1, 1, (X.shape[0], 3))
    Xd, Fd = torch.from_numpy(X).to(dev), torch.from_numpy(F).to(dev)
    idd, xsd = torch.from_numpy(idx).to(dev), torch.from_numpy(xs).to(dev)
    m = le.Markers(ctx).bin(geom, kernel, Xd, idd, xsd)
    Q = torch.zeros((X.shape[0], 3), dtype=torch.float64, device=dev)
    le.interp(ctx, m, kernel, "side", geom, q, Q, Xd)
    le.spread(ctx, m, kernel, "side", geom, q, Fd, Xd)
    ctx.synchronize()
    order = m.order().cpu().numpy()
    Qo = np.zeros((X.shape[0], 3))
    oracle.side_interp(kernel, geom.dx, geom.x_lower, geom.ilower, geom.iupper, geom.gcw, u0, idx, xs, X, Qo)
    uo = [a.copy() for a in u0]
    oracle.side_spread(kernel, geom.dx, geom.x_lower, geom.ilower, geom.iupper, geom.gcw, uo, idx[order],
                       xs[order], X, F)
    assert np.array_equal(Q.cpu().numpy()[idx], Qo[idx])
    # and against the reference's own summation order: the caller's list order
    uc = [a.copy() for a in u0]
    oracle.side_spread(kernel, geom.dx, geom.x_lower, geom.ilower, geom.iupper, geom.gcw, uc, idx, xs, X, F)
    for a in range(3):
        ga = q[a].cpu().numpy()
        assert np.abs(ga - uo[a]).max() <= SPREAD_TOL * np.abs(uo[a]).max()
        assert np.abs(ga - uc[a]).max() <= SPREAD_TOL * np.abs(uc[a]).max(), f"comp {a} vs caller order"


def test_spread_bit_stable_run_to_run(le, ctx):
    """Same inputs, two runs (and a re-bin in between): identical bits."""
    from ibamr_amd.le import Geometry
    geom = Geometry.periodic_unit([48, 48, 48], 3)
    g = torch.Generator(device="cuda:0").manual_seed(9)
    M = 200_000
    X = torch.rand((M, 3), dtype=torch.float64, device="cuda:0", generator=g)
    F = torch.rand((M, 3), dtype=torch.float64, device="cuda:0", generator=g) - 0.5
    outs = []
    for rep in range(2):
        q = geom.alloc("side")
        m = le.Markers(ctx).bin(geom, "IB_4", X)
        le.spread(ctx, m, "IB_4", "side", geom, q, F, X)
        ctx.synchronize()
        outs.append([a.clone() for a in q])
    for a in range(3):
        assert torch.equal(outs[0][a], outs[1][a])


@pytest.mark.parametrize("kernel", ["IB_4", "IB_6", "PIECEWISE_CONSTANT"])
def test_spread_bit_stable_dense(le, ctx, oracle, kernel):
    """Many markers per cell (shared stencil starts, so one add instruction
    carries several lanes to the same grid point): still bit-stable, and within
    tolerance of the oracle."""
    from ibamr_amd.le import Geometry
    geom = Geometry.periodic_unit([24, 24, 24], oracle.min_ghost_width(kernel) + 1)
    g = torch.Generator(device="cuda:0").manual_seed(4)
    M = 60_000
    X = 0.40 + 0.05 * torch.rand((M, 3), dtype=torch.float64, device="cuda:0", generator=g)
    X[: M // 2] = X[0]  # half the markers at one point
    F = torch.rand((M, 3), dtype=torch.float64, device="cuda:0", generator=g) - 0.5
    outs = []
    for rep in range(2):
        q = geom.alloc("side")
        m = le.Markers(ctx).bin(geom, kernel, X)
        le.spread(ctx, m, kernel, "side", geom, q, F, X)
        ctx.synchronize()
        outs.append([a.clone() for a in q])
    for a in range(3):
        assert torch.equal(outs[0][a], outs[1][a])
    order = m.order().cpu().numpy()
    idx = np.arange(M, dtype=np.int32)
    uo = [np.zeros(tuple(a.shape)) for a in outs[0]]
    oracle.side_spread(kernel, geom.dx, geom.x_lower, geom.ilower, geom.iupper, geom.gcw, uo, idx[order],
                       np.zeros((M, 3)), X.cpu().numpy(), F.cpu().numpy())
    for a in range(3):
        ga = outs[0][a].cpu().numpy()
        assert np.abs(ga - uo[a]).max() <= SPREAD_TOL * np.abs(uo[a]).max()


def test_errors_are_reported(le, ctx):
    from ibamr_amd._lib import IBTKLEError
    from ibamr_amd.le import Geometry
    geom = Geometry.periodic_unit([16, 16, 16], 2)  # too few ghosts for IB_4 interp
    X = torch.rand((10, 3), dtype=torch.float64, device="cuda:0")
    q = geom.alloc("side")
    Q = torch.zeros((10, 3), dtype=torch.float64, device="cuda:0")
    m = le.Markers(ctx).bin(geom, "IB_4", X)
    with pytest.raises(IBTKLEError) as e:
        le.interp(ctx, m, "IB_4", "side", geom, q, Q, X)
    assert e.value.code == 2
    with pytest.raises(IBTKLEError) as e:
        le.Markers(ctx).bin(geom, "NOT_A_KERNEL", X)
    assert e.value.code == 1
    with pytest.raises(IBTKLEError) as e:  # side data needs Q depth NDIM
        le.spread(ctx, m, "IB_4", "side", geom, q, Q[:, :2].contiguous(), X, Q_depth=2)
    assert e.value.code == 3


def test_empty_list_is_a_noop(le, ctx):
    from ibamr_amd.le import Geometry
    geom = Geometry.periodic_unit([16, 16, 16], 3)
    X = torch.zeros((0, 3), dtype=torch.float64, device="cuda:0")
    q = geom.alloc("side", fill=1.5)
    m = le.Markers(ctx).bin(geom, "IB_4", X)
    le.spread(ctx, m, "IB_4", "side", geom, q, X, X)
    le.interp(ctx, m, "IB_4", "side", geom, q, X, X)
    ctx.synchronize()
    assert all(bool((a == 1.5).all()) for a in q)


@pytest.mark.parametrize("kernel", ALL)
def test_dense_uniform_side(le, ctx, oracle, kernel):
    """~2 markers per cell: hundreds of markers per (column, anchor plane), so
    the sweeps run full middle chunks and carry leftovers from one anchor plane
    into the next; interp bitwise-close and spread within tolerance of the oracle."""
    from ibamr_amd.le import Geometry
    geom = Geometry.periodic_unit([32, 32, 32], oracle.min_ghost_width(kernel) + 1)
    g = torch.Generator(device="cuda:0").manual_seed(21)
    M = 65_000
    X = torch.rand((M, 3), dtype=torch.float64, device="cuda:0", generator=g)
    F = torch.rand((M, 3), dtype=torch.float64, device="cuda:0", generator=g) - 0.5
    u = geom.alloc("side")
    for a in u:
        a.uniform_(-1.0, 1.0, generator=g)
    le.fill_periodic_ghosts(ctx, geom, "side", u)
    u0 = [a.cpu().numpy().copy() for a in u]
    U = torch.zeros((M, 3), dtype=torch.float64, device="cuda:0")
    m = le.Markers(ctx).bin(geom, kernel, X)
    le.interp(ctx, m, kernel, "side", geom, u, U, X)
    q = geom.alloc("side")
    le.spread(ctx, m, kernel, "side", geom, q, F, X)
    ctx.synchronize()
    Xn, Fn = X.cpu().numpy(), F.cpu().numpy()
    idx = np.arange(M, dtype=np.int32)
    xs = np.zeros((M, 3))
    Uo = np.zeros((M, 3))
    oracle.side_interp(kernel, geom.dx, geom.x_lower, geom.ilower, geom.iupper, geom.gcw, u0, idx, xs, Xn, Uo)
    assert rel_err(U.cpu().numpy(), Uo) <= INTERP_TOL
    order = m.order().cpu().numpy()
    uo = [np.zeros(tuple(a.shape)) for a in q]
    oracle.side_spread(kernel, geom.dx, geom.x_lower, geom.ilower, geom.iupper, geom.gcw, uo, idx[order], xs, Xn, Fn)
    for a in range(3):
        assert rel_err(q[a].cpu().numpy(), uo[a]) <= SPREAD_TOL, f"spread comp {a}"


@pytest.mark.parametrize("kernel", ["IB_4", "IB_6", "BSPLINE_4"])
def test_vertex_file_sphere(le, ctx, oracle, kernel):
    """Markers from a reference input deck (tests/golden/vertex/sphere3d_32.vertex,
    read by ibamr_amd.io as IBStandardInitializer would, scaled to radius 0.125 about
    the box centre): interp and spread against the oracle."""
    import os
    from ibamr_amd import io
    from ibamr_amd.le import Geometry
    Xn = io.read_vertex(os.path.join(os.path.dirname(__file__), "golden", "vertex", "sphere3d_32.vertex"),
                        length_scale=0.25, posn_shift=[2.0, 2.0, 2.0])
    M = Xn.shape[0]
    geom = Geometry.periodic_unit([32, 32, 32], oracle.min_ghost_width(kernel))
    rng = np.random.default_rng(4)
    Fn = rng.standard_normal((M, 3))
    u = geom.alloc("side")
    for a in u:
        a.copy_(torch.from_numpy(rng.standard_normal(tuple(a.shape))))
    u0 = [a.cpu().numpy().copy() for a in u]
    X = torch.from_numpy(Xn).cuda()
    F = torch.from_numpy(Fn).cuda()
    U = torch.zeros((M, 3), dtype=torch.float64, device="cuda:0")
    m = le.Markers(ctx).bin(geom, kernel, X)
    le.interp(ctx, m, kernel, "side", geom, u, U, X)
    q = geom.alloc("side")
    le.spread(ctx, m, kernel, "side", geom, q, F, X)
    ctx.synchronize()
    idx = np.arange(M, dtype=np.int32)
    xs = np.zeros((M, 3))
    Uo = np.zeros((M, 3))
    oracle.side_interp(kernel, geom.dx, geom.x_lower, geom.ilower, geom.iupper, geom.gcw, u0, idx, xs, Xn, Uo)
    assert rel_err(U.cpu().numpy(), Uo) <= INTERP_TOL
    order = m.order().cpu().numpy()
    uo = [np.zeros(tuple(a.shape)) for a in q]
    oracle.side_spread(kernel, geom.dx, geom.x_lower, geom.ilower, geom.iupper, geom.gcw, uo, idx[order], xs, Xn, Fn)
    for a in range(3):
        assert rel_err(q[a].cpu().numpy(), uo[a]) <= SPREAD_TOL, f"spread comp {a}"


@pytest.mark.parametrize("kernel", ["IB_4", "BSPLINE_4", "IB_6"])
def test_spread_at_rounding_ties(le, ctx, oracle, kernel):
    """Markers where (X - xlo) * (1/dx) and (X - xlo) / dx round to different NINT
    anchors (the spread stencil multiplies, the bin key divides): the stencil can
    move one cell, onto a point whose weight is of an ulp's order, so the spread
    still matches the oracle (which divides, as the Fortran does) within tolerance."""
    from ibamr_amd.le import Geometry
    dx, xlo, N = 0.1, -0.3, 14
    geom = Geometry([0, 0, 0], [N - 1] * 3, oracle.min_ghost_width(kernel), [dx] * 3, [xlo] * 3)
    ties = []
    for k in range(2, N - 2):
        base = xlo + (k + 0.5) * dx
        for j in range(-40, 41):
            X = base + j * np.spacing(base)
            if np.floor((X - xlo) * (1.0 / dx) + 0.5) != np.floor((X - xlo) / dx + 0.5):
                ties.append(X)
    ties = np.array(ties)
    assert ties.size >= 4
    rng = np.random.default_rng(2)
    M = 600
    Xn = rng.choice(ties, size=(M, 3))
    Fn = rng.standard_normal((M, 3))
    X, F = torch.from_numpy(Xn).cuda(), torch.from_numpy(Fn).cuda()
    m = le.Markers(ctx).bin(geom, kernel, X)
    q = geom.alloc("side")
    le.spread(ctx, m, kernel, "side", geom, q, F, X)
    ctx.synchronize()
    order = m.order().cpu().numpy()
    uo = [np.zeros(tuple(a.shape)) for a in q]
    oracle.side_spread(kernel, geom.dx, geom.x_lower, geom.ilower, geom.iupper, geom.gcw, uo,
                       np.arange(M, dtype=np.int32)[order], np.zeros((M, 3)), Xn, Fn)
    for a in range(3):
        assert rel_err(q[a].cpu().numpy(), uo[a]) <= SPREAD_TOL, f"spread comp {a}"
