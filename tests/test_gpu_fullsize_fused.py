"""GPU: the exact fused paths bench.py times, at BASELINE.json's full sizes (VERDICT r4,
"Next round" item 4), through size-independent properties:

* cfg4 (1024^3, 1e8 uniform markers, IB_4): ibtk_le_zero_spread into an f full of NaN
  (every point written, none read) equals the zeroing followed by ibtk_le_spread, bit for
  bit, and run to run; ibtk_le_fill_interp with NaN ghosts (no ghost point read)
  equals the periodic fill followed by ibtk_le_interp, bit for bit; conservation,
  adjointness and the constant field through the fused calls.
* cfg5 (a 512^3 level of 8^3 patches of 64^3, 1e7 clustered markers): the level's
  fused zero + spread and ghost fill + interp (ibtk_le_level_zero_spread,
  ibtk_le_level_fill_interp) against the unfused pairs, bit for bit, with NaN ghosts
  and a NaN f; conservation over the patches' unique points and adjointness between
  the interior lists' interp and the ghost-box lists' spread.
* cfg4 moving: one explicit step's displacement (5 % of a cell, bench.py --move), then
  ibtk_le_markers_rebin against a fresh binning at 1024^3: the same order, and the
  fused interp and spread through either bit for bit.
The sums run in fp64 over 1e7-1e9 terms; the 1e-10 relative tolerances bound their
rounding, not the kernels'.
"""
import math

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


def _unique(t, g, n):
    return t[g:g + n, g:g + n, g:g + n]


def _nan_ghosts(t, g, n):
    """NaN on every ghost point (and on a side array's upper face, the periodic copy of its
    lower one): what a fused fill must not read."""
    keep = _unique(t, g, n).clone()
    t.fill_(float("nan"))
    _unique(t, g, n).copy_(keep)


def test_cfg4_fused_paths_fullsize(le, ctx):
    N, M, kernel = 1024, 100_000_000, "IB_4"
    g = le._lib.load().ibtk_le_min_ghost_width(le.kernel_id(kernel))
    geom = le.Geometry.periodic_unit([N] * 3, ghost=g)
    h3 = geom.dx[0] * geom.dx[1] * geom.dx[2]
    gen = torch.Generator(device="cuda").manual_seed(1234)
    X = torch.rand((M, 3), dtype=torch.float64, device="cuda", generator=gen)
    F = torch.rand((M, 3), dtype=torch.float64, device="cuda", generator=gen) * 2 - 1
    m = le.Markers(ctx).bin(geom, kernel, X)
    # spread: the fused form into a NaN f, twice, and the unfused pair
    f = geom.alloc("side")
    for t in f:
        t.fill_(float("nan"))
    le.zero_spread(ctx, m, kernel, "side", geom, f, F, X)
    f2 = geom.alloc("side")
    for t in f2:
        t.fill_(float("nan"))
    le.zero_spread(ctx, m, kernel, "side", geom, f2, F, X)
    ctx.synchronize()
    for a in range(3):
        assert not torch.isnan(f[a]).any(), f"component {a}: a point of f left unwritten"
        assert torch.equal(f[a], f2[a]), f"component {a}: zero_spread not bit-stable"
    for t in f2:
        t.zero_()
    le.spread(ctx, m, kernel, "side", geom, f2, F, X)
    ctx.synchronize()
    for a in range(3):
        assert torch.equal(f[a], f2[a]), f"component {a}: zero_spread differs from zero + spread"
    del f2
    le.fold_periodic_ghosts(ctx, geom, "side", f)
    ctx.synchronize()
    for a in range(3):
        tot = _unique(f[a], g, N).sum().item() * h3
        assert abs(tot - F[:, a].sum().item()) <= 1e-10 * F[:, a].abs().sum().item(), a
    # interp: the fused fill with NaN ghosts, against the fill then interp
    u = geom.alloc("side")
    for t in u:
        t.uniform_(-1, 1, generator=gen)
        _nan_ghosts(t, g, N)
    Q1 = torch.empty_like(F)
    le.fill_interp(ctx, m, kernel, "side", geom, u, Q1, X)
    le.fill_periodic_ghosts(ctx, geom, "side", u)
    Q2 = torch.empty_like(F)
    le.interp(ctx, m, kernel, "side", geom, u, Q2, X)
    ctx.synchronize()
    assert not torch.isnan(Q1).any(), "fill_interp read a ghost point"
    assert torch.equal(Q1, Q2)
    lhs = (Q1 * F).sum().item()
    rhs = h3 * sum((_unique(u[a], g, N) * _unique(f[a], g, N)).sum().item() for a in range(3))
    assert abs(lhs - rhs) <= 1e-10 * (Q1.abs() * F.abs()).sum().item(), (lhs, rhs)
    del Q2, f
    for t in u:
        t.fill_(0.75)
        _nan_ghosts(t, g, N)
    le.fill_interp(ctx, m, kernel, "side", geom, u, Q1, X)
    ctx.synchronize()
    assert (Q1 - 0.75).abs().max().item() <= 1e-14
    del u, Q1, X, F, m
    torch.cuda.empty_cache()


def test_cfg5_level_fused_paths_fullsize(le, ctx):
    import bench
    from ibamr_amd.slab import Slab
    cfg = bench.CONFIGS["cfg5"]
    N, P, M, kernel = cfg["N"], cfg["patches"], cfg["M"], cfg["kernel"]
    n = N // P
    g = le._lib.load().ibtk_le_min_ghost_width(le.kernel_id(kernel))
    dx = 1.0 / N
    h3 = dx ** 3
    geoms = []
    for k in range(P):
        for j in range(P):
            for i in range(P):
                lo = [i * n, j * n, k * n]
                geoms.append(le.Geometry(lo, [v + n - 1 for v in lo], g, [dx] * 3, [v * dx for v in lo]))
    X = bench.make_markers("clustered", M, Slab([N, N, N], 1, 0, g), 1234, "cuda")
    X = torch.remainder(X, 1.0).contiguous()
    M = X.shape[0]
    gen = torch.Generator(device="cuda").manual_seed(4321)
    F = torch.rand((M, 3), dtype=torch.float64, device="cuda", generator=gen) * 2 - 1
    (ii, _, oi), (si, sx, os_) = bench.level_lists(X, N, P, g)
    lvl = le.Level.from_flat(ctx, geoms, kernel, X, si, sx, os_)
    lvl.select_interior(M, ii, oi)
    # spread: fused into NaN arrays, twice, against zero + spread
    f = le.alloc_level(geoms, "side")
    for per in f:
        for t in per:
            t.fill_(float("nan"))
    lvl.zero_spread("side", f, F, X)
    f2 = le.alloc_level(geoms, "side")
    for per in f2:
        for t in per:
            t.fill_(float("nan"))
    lvl.zero_spread("side", f2, F, X)
    ctx.synchronize()
    for q in range(len(geoms)):
        for a in range(3):
            assert not torch.isnan(f[q][a]).any(), (q, a)
            assert torch.equal(f[q][a], f2[q][a]), (q, a)
    lvl.zero("side", f2)
    lvl.spread("side", f2, F, X)
    ctx.synchronize()
    for q in range(len(geoms)):
        for a in range(3):
            assert torch.equal(f[q][a], f2[q][a]), (q, a)
    del f2
    # conservation over the unique points of every patch (each marker's stencil lands in
    # the patches owning its points through the ghost-box lists' entries and images)
    for a in range(3):
        tot = sum(_unique(f[q][a], g, n).sum().item() for q in range(len(geoms))) * h3
        assert abs(tot - F[:, a].sum().item()) <= 1e-10 * F[:, a].abs().sum().item(), a
    # interp: the fused level fill with NaN ghosts, against the fill then interp
    u = le.alloc_level(geoms, "side")
    for per in u:
        for t in per:
            t.uniform_(-1, 1, generator=gen)
            _nan_ghosts(t, g, n)
    Q1 = torch.empty_like(F)
    lvl.fill_interp("side", u, Q1, X)
    lvl.fill_ghosts("side", u)
    Q2 = torch.empty_like(F)
    lvl.interp("side", u, Q2, X)
    ctx.synchronize()
    assert not torch.isnan(Q1).any(), "level fill_interp read an unfilled ghost point"
    assert torch.equal(Q1, Q2)
    # adjointness: the interior lists' interp (each marker once) against the ghost-box
    # lists' spread, over the unique points
    lhs = (Q1 * F).sum().item()
    rhs = h3 * sum((_unique(u[q][a], g, n) * _unique(f[q][a], g, n)).sum().item()
                   for q in range(len(geoms)) for a in range(3))
    assert abs(lhs - rhs) <= 1e-10 * (Q1.abs() * F.abs()).sum().item(), (lhs, rhs)
    del u, f, Q1, Q2, lvl, X, F
    torch.cuda.empty_cache()


def test_cfg4_rebin_after_moving_step_fullsize(le, ctx):
    N, M, kernel = 1024, 100_000_000, "IB_4"
    g = le._lib.load().ibtk_le_min_ghost_width(le.kernel_id(kernel))
    geom = le.Geometry.periodic_unit([N] * 3, ghost=g)
    gen = torch.Generator(device="cuda").manual_seed(99)
    X = torch.rand((M, 3), dtype=torch.float64, device="cuda", generator=gen)
    F = torch.rand((M, 3), dtype=torch.float64, device="cuda", generator=gen) * 2 - 1
    m = le.Markers(ctx).bin(geom, kernel, X)
    # one explicit step of bench.py --move: X += dt U, |U| <= 1, dt = cell / 20
    U = torch.rand((M, 3), dtype=torch.float64, device="cuda", generator=gen) * 2 - 1
    le.position_update(ctx, "euler", 0.05 * geom.dx[0], X, U, out=X)
    X.remainder_(1.0)
    del U
    m.rebin(X)
    fresh = le.Markers(ctx).bin(geom, kernel, X)
    assert torch.equal(m.order(), fresh.order())
    u = geom.alloc("side")
    for t in u:
        t.uniform_(-1, 1, generator=gen)
    Q1, Q2 = torch.empty_like(F), torch.empty_like(F)
    le.fill_interp(ctx, m, kernel, "side", geom, u, Q1, X)
    le.fill_interp(ctx, fresh, kernel, "side", geom, u, Q2, X)
    ctx.synchronize()
    assert torch.equal(Q1, Q2)
    del u, Q1, Q2
    f1, f2 = geom.alloc("side"), geom.alloc("side")
    le.zero_spread(ctx, m, kernel, "side", geom, f1, F, X)
    le.zero_spread(ctx, fresh, kernel, "side", geom, f2, F, X)
    ctx.synchronize()
    for a in range(3):
        assert torch.equal(f1[a], f2[a]), a
    del f1, f2, X, F, m, fresh
    torch.cuda.empty_cache()
