"""GPU: a spread's bits depend on the binning, not on which spreads ran since it (advisor,
round 5).

The 3-D spread's candidate stream is built on the first spread after a binning and kept.
A closed-form kernel's stream is split by the shifted-z anchor (the z-side component's
frame), which reorders each column-anchor's candidates -- the order in which they add into
a point.  It is now split whatever the first spread's centering was, so a cell-centred
spread run after a side-centred one on the same binning equals the same spread on a fresh
binning bit for bit, and the other way round."""
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


def _spread(le, ctx, m, kernel, centering, geom, F, X, depth):
    q = geom.alloc(centering, depth=depth)
    le.spread(ctx, m, kernel, centering, geom, q, F, X, q_depth=depth)
    ctx.synchronize()
    return q


@pytest.mark.parametrize("kernel", ["IB_4", "IB_6"])
@pytest.mark.parametrize("first,second", [("side", "cell"), ("cell", "side"), ("node", "cell")])
def test_spread_bits_do_not_depend_on_earlier_spreads(le, kernel, first, second):
    g = le._lib.load().ibtk_le_min_ghost_width(le.kernel_id(kernel))
    geom = le.Geometry.periodic_unit([64, 48, 40], g)
    rng = np.random.default_rng(11)
    M = 30000
    X = torch.from_numpy(rng.uniform(0.0, 1.0, (M, 3))).cuda()
    F = torch.from_numpy(rng.standard_normal((M, 3))).cuda()
    depth = {"side": 1, "cell": 3, "node": 3}
    ctx = le.Context(0)
    m = le.Markers(ctx).bin(geom, kernel, X)
    _spread(le, ctx, m, kernel, first, geom, F, X, depth[first])
    after = _spread(le, ctx, m, kernel, second, geom, F, X, depth[second])
    fresh = _spread(le, ctx, le.Markers(ctx).bin(geom, kernel, X), kernel, second, geom, F, X, depth[second])
    for a, b in zip(after, fresh):
        assert torch.equal(a, b)
    # and after a re-binning that moved markers (the stream rebuilt from the new order)
    h = 1.0 / 64
    X2 = torch.remainder(X + 0.4 * h * (torch.rand_like(X) - 0.5), 1.0)
    m.rebin(X2)
    _spread(le, ctx, m, kernel, first, geom, F, X2, depth[first])
    after = _spread(le, ctx, m, kernel, second, geom, F, X2, depth[second])
    fresh = _spread(le, ctx, le.Markers(ctx).bin(geom, kernel, X2), kernel, second, geom, F, X2, depth[second])
    for a, b in zip(after, fresh):
        assert torch.equal(a, b)


def test_select_interior_lists_changed_in_place(le):
    """Level.select_interior(lists_changed=True) (or reset_selection()) recomputes a selection
    whose int32 interior list was rewritten in place; the interp then matches a fresh level."""
    import bench
    from ibamr_amd.slab import Slab
    N, P = 64, 2
    n = N // P
    g = le._lib.load().ibtk_le_min_ghost_width(le.kernel_id("IB_4"))
    geoms = []
    for k in range(P):
        for j in range(P):
            for i in range(P):
                lo = [i * n, j * n, k * n]
                geoms.append(le.Geometry(lo, [v + n - 1 for v in lo], g, [1.0 / N] * 3, [v / N for v in lo]))
    ctx = le.Context(0)
    X = bench.make_markers("uniform", 20000, Slab([N, N, N], 1, 0, g), 3, "cuda")
    X = torch.remainder(X, 1.0).contiguous()
    M = X.shape[0]
    (ii, _, oi), (si, sx, os_) = bench.level_lists(X, N, P, g)
    u = le.alloc_level(geoms, "side")
    for per in u:
        for a in per:
            a.uniform_(-1.0, 1.0)
    lvl = le.Level.from_flat(ctx, geoms, "IB_4", X, si, sx, os_)
    ii32 = ii.to(torch.int32).contiguous()
    lvl.select_interior(M, ii32, oi)
    U0 = torch.zeros((M, 3), dtype=torch.float64, device="cuda")
    lvl.fill_ghosts("side", u)
    lvl.interp("side", u, U0, X)
    # rewrite the interior list in place: swap a marker A of patch 0 near its +x face with a
    # marker B of patch 1 near the same face (each lies in the other patch's ghost box, so
    # the lists stay valid): A's Q now comes from patch 1's arrays and B's from patch 0's,
    # where a kept, stale selection would still take them from their old patches
    cellx = torch.floor(X[:, 0] * N).long()
    e0 = torch.arange(oi[0], oi[1], device="cuda")
    e1 = torch.arange(oi[1], oi[2], device="cuda")
    ea = e0[cellx[ii32[e0].long()] == n - 1][0]
    eb = e1[cellx[ii32[e1].long()] == n][0]
    A, B = int(ii32[ea].item()), int(ii32[eb].item())
    ii32[ea] = B
    ii32[eb] = A
    oi2 = list(oi)
    for fresh_sel in (False, True):
        lvl2 = le.Level.from_flat(ctx, geoms, "IB_4", X, si, sx, os_)
        lvl2.select_interior(M, ii32.clone(), oi2)
        U_ref = torch.full((M, 3), 7.0, dtype=torch.float64, device="cuda")
        lvl2.interp("side", u, U_ref, X)
        U1 = torch.full((M, 3), 7.0, dtype=torch.float64, device="cuda")
        if fresh_sel:
            lvl.reset_selection()
            lvl.select_interior(M, ii32, oi2)
        else:
            lvl.select_interior(M, ii32, oi2, lists_changed=True)
        lvl.interp("side", u, U1, X)
        ctx.synchronize()
        assert torch.equal(U1, U_ref)


@pytest.mark.parametrize("kernel", ["IB_4", "IB_6"])
def test_side_stream_gather_matches_in_line(le, kernel):
    """The spread's F gather runs on the context's side stream while the candidate stream
    is rebuilt (ibtk_le_ctx_tune "side_gather" 1; by default from 2^25 markers); it sees F as the caller's
    stream left it just before the call (here rewritten in place between spreads) and the
    result equals the in-line gather's (-1) bit for bit, on the first spread after a
    binning, after a re-binning that moved markers, and on a standing stream."""
    g = le._lib.load().ibtk_le_min_ghost_width(le.kernel_id(kernel))
    geom = le.Geometry.periodic_unit([64, 48, 40], g)
    rng = np.random.default_rng(5)
    M = 40000
    X = torch.from_numpy(rng.uniform(0.0, 1.0, (M, 3))).cuda()
    F0 = torch.from_numpy(rng.standard_normal((M, 3))).cuda()
    h = 1.0 / 64
    X2 = torch.remainder(X + 0.4 * h * (torch.rand_like(X) - 0.5), 1.0)
    outs = {}
    for mode in (-1, 1):
        ctx = le.Context(0)
        ctx.tune("side_gather", mode)
        F = F0.clone()
        m = le.Markers(ctx).bin(geom, kernel, X)
        res = [_spread(le, ctx, m, kernel, "side", geom, F, X, 1)]
        F.mul_(-0.75).add_(0.125)          # F changes every step
        m.rebin(X2)
        res.append(_spread(le, ctx, m, kernel, "side", geom, F, X2, 1))
        F.mul_(1.5)
        res.append(_spread(le, ctx, m, kernel, "side", geom, F, X2, 1))  # standing stream
        outs[mode] = res
    for a, b in zip(outs[-1], outs[1]):
        for x, y in zip(a, b):
            assert torch.equal(x, y)
    # and the second spread is not the first one's F: the gather saw the rewrite
    assert not torch.equal(outs[1][1][0], outs[1][0][0])
