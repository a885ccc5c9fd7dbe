"""GPU: the incremental re-binning (ibtk_le_markers_rebin) equals a fresh binning.

Rebin takes the previous sorted order of the same list and inserts the entries
whose bucket changed.  The order by (bucket, list entry) is unique, so the result
must be the fresh binning's exactly: the same canonical order, and interp / spread
through the rebinned list bitwise equal to the freshly binned one (that covers the
sorted positions, the bucket starts and the sweep item table).  Cases: nothing
moved, small moves (a fraction of the markers change bucket), every marker moved,
a sheet crossing a plane together (long per-bucket mover lists), markers leaving
and re-entering the patch, index lists with periodic shifts, a level of patches,
and repeated re-binnings (the device counters clean up after themselves)."""
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


def _fields(le, geom, rng):
    u = geom.alloc("side")
    for a in u:
        a.copy_(torch.from_numpy(rng.uniform(-1, 1, tuple(a.shape))))
    return u


def _run(le, ctx, m, geom, u, X, F, kernel="IB_4"):
    M = F.shape[0]
    U = torch.zeros((M, 3), dtype=torch.float64, device="cuda")
    le.interp(ctx, m, kernel, "side", geom, u, U, X)
    f = geom.alloc("side")
    le.spread(ctx, m, kernel, "side", geom, f, F, X)
    ctx.synchronize()
    return U, f


def _check_same(le, geom, ctx, m_re, X, F, u, kernel="IB_4", indices=None, xshift=None):
    """m_re (rebinned at X) against a fresh binning of the same list at X."""
    m_fr = le.Markers(ctx).bin(geom, kernel, X, indices, xshift)
    assert torch.equal(m_re.order(), m_fr.order())
    U1, f1 = _run(le, ctx, m_re, geom, u, X, F, kernel)
    U2, f2 = _run(le, ctx, m_fr, geom, u, X, F, kernel)
    assert torch.equal(U1, U2)
    for a, b in zip(f1, f2):
        assert torch.equal(a, b)


@pytest.mark.parametrize("kernel", ["IB_4", "IB_6", "PIECEWISE_LINEAR"])
def test_rebin_equals_fresh_bin(le, kernel):
    N = (96, 64, 80)
    geom = le.Geometry.periodic_unit(list(N), le._lib.load().ibtk_le_min_ghost_width(le.kernel_id(kernel)))
    rng = np.random.default_rng(5)
    M = 40000
    X = torch.from_numpy(rng.uniform(0.0, 1.0, (M, 3))).cuda()
    F = torch.from_numpy(rng.standard_normal((M, 3))).cuda()
    u = _fields(le, geom, rng)
    ctx = le.Context(0)
    m = le.Markers(ctx).bin(geom, kernel, X)
    # nothing moved
    m.rebin(X)
    _check_same(le, geom, ctx, m, X, F, u, kernel)
    # small moves, three steps in a row (a fraction change bucket each step)
    h = torch.tensor([1.0 / n for n in N], dtype=torch.float64, device="cuda")
    for step in range(3):
        X = torch.remainder(X + 0.3 * h * (torch.rand_like(X) - 0.5), 1.0)
        m.rebin(X)
        _check_same(le, geom, ctx, m, X, F, u, kernel)
    # every marker somewhere else
    X = torch.from_numpy(rng.uniform(0.0, 1.0, (M, 3))).cuda()
    m.rebin(X)
    _check_same(le, geom, ctx, m, X, F, u, kernel)


def test_rebin_sheet_crossing_a_plane(le):
    """A one-cell sheet moving half a cell in z: thousands of movers into the same
    buckets (the long-list sort of k_rebin_sort_big), plus markers leaving the
    patch (outside key) and coming back."""
    N = (64, 64, 64)
    geom = le.Geometry((0, 0, 0), (63, 63, 63), 3, [1.0 / 64] * 3, [0.0, 0.0, 0.0])
    rng = np.random.default_rng(9)
    M = 60000
    Xn = rng.uniform(0.0, 1.0, (M, 3))
    Xn[: 40000, 2] = 0.5 + (Xn[: 40000, 2] - 0.5) / 64.0 * 0.2       # the sheet
    Xn[: 40000, 0] = 0.40 + 0.05 * Xn[: 40000, 0]                     # dense in a few columns
    X = torch.from_numpy(Xn).cuda()
    F = torch.from_numpy(rng.standard_normal((M, 3))).cuda()
    u = _fields(le, geom, rng)
    ctx = le.Context(0)
    m = le.Markers(ctx).bin(geom, "IB_4", X)
    X2 = X.clone()
    X2[: 40000, 2] += 0.5 / 64
    X2[40000: 41000, 0] = 1.5   # out of the patch (and its ghost box): binned outside
    m.rebin(X2)
    _check_same(le, geom, ctx, m, X2, F, u)
    m.rebin(X)                   # and back
    _check_same(le, geom, ctx, m, X, F, u)


def test_rebin_index_list_with_shifts(le):
    """A periodic index list (entries with Xshift): rebin keeps the list, moves the
    markers."""
    N = (48, 40, 56)
    geom = le.Geometry.periodic_unit(list(N), 3)
    rng = np.random.default_rng(13)
    M = 20000
    X = torch.from_numpy(rng.uniform(0.0, 1.0, (M, 3))).cuda()
    ctx = le.Context(0)
    idx, xs = le.periodic_index_list(ctx, geom, X, 3)
    n = idx.numel()
    F = torch.from_numpy(rng.standard_normal((M, 3))).cuda()
    u = _fields(le, geom, rng)
    m = le.Markers(ctx).bin(geom, "IB_4", X, idx, xs)
    h = 1.0 / 48
    X2 = X + 0.4 * h * (torch.rand_like(X) - 0.5)   # stays within the ghost slack of the list
    m.rebin(X2)
    _check_same(le, geom, ctx, m, X2, F, u, indices=idx, xshift=xs)
    assert m.count() == n


def test_rebin_level(le):
    """A level of 2^3 patches: rebin of the level's lists equals a fresh level bin."""
    N, P = 64, 2
    n = N // P
    g = 3
    geoms = []
    for k in range(P):
        for j in range(P):
            for i in range(P):
                lo = [i * n, j * n, k * n]
                geoms.append(le.Geometry(lo, [v + n - 1 for v in lo], g, [1.0 / N] * 3, [v / N for v in lo]))
    rng = np.random.default_rng(17)
    M = 30000
    X = torch.from_numpy(rng.uniform(0.0, 1.0, (M, 3))).cuda()
    ctx = le.Context(0)
    c = torch.clamp((X * N).floor().long(), 0, N - 1) // n
    pid = (c[:, 2] * P + c[:, 1]) * P + c[:, 0]
    lists = [(torch.nonzero(pid == q).flatten().to(torch.int32), None) for q in range(P ** 3)]
    lvl = le.Level(ctx, geoms, "IB_4", X, lists)
    u = [_fields(le, gq, rng) for gq in geoms]
    F = torch.from_numpy(rng.standard_normal((M, 3))).cuda()
    X2 = X + (0.6 / N) * (torch.rand_like(X) - 0.5)
    lvl.rebin(X2)
    fresh = le.Level(ctx, geoms, "IB_4", X2, lists)
    assert torch.equal(lvl.markers.order(), fresh.markers.order())
    outs = []
    for L in (lvl, fresh):
        U = torch.zeros((M, 3), dtype=torch.float64, device="cuda")
        L.interp("side", u, U, X2)
        f = [gq.alloc("side") for gq in geoms]
        L.spread("side", f, F, X2)
        ctx.synchronize()
        outs.append((U, f))
    assert torch.equal(outs[0][0], outs[1][0])
    for fa, fb in zip(outs[0][1], outs[1][1]):
        for a, b in zip(fa, fb):
            assert torch.equal(a, b)


def test_rebin_empty_and_tiny(le):
    geom = le.Geometry.periodic_unit([32, 32, 32], 3)
    ctx = le.Context(0)
    rng = np.random.default_rng(1)
    for M in (0, 1, 33):
        X = torch.from_numpy(rng.uniform(0.0, 1.0, (M, 3))).cuda()
        F = torch.from_numpy(rng.standard_normal((M, 3))).cuda()
        u = _fields(le, geom, rng)
        m = le.Markers(ctx).bin(geom, "IB_4", X)
        X2 = torch.from_numpy(rng.uniform(0.0, 1.0, (M, 3))).cuda()
        m.rebin(X2)
        if M:
            _check_same(le, geom, ctx, m, X2, F, u)


def test_rebin_after_bin_count_keeps_its_count(le):
    """a rebin after bin_count reads the count again on the device;
    the Python wrapper keeps the count tensor alive, and the rebin equals a fresh
    count-binning even after the caller dropped its reference and the allocator reused
    the memory."""
    import gc
    N = (48, 48, 64)
    geom = le.Geometry.periodic_unit(list(N), 3)
    rng = np.random.default_rng(12)
    cap, M = 12000, 10000
    X = torch.zeros((cap, 3), dtype=torch.float64, device="cuda")
    X[:M] = torch.from_numpy(rng.uniform(0.0, 1.0, (M, 3))).cuda()
    ctx = le.Context(0)
    m = le.Markers(ctx).bin_count(geom, "IB_4", X, torch.tensor([M], dtype=torch.int32, device="cuda"))
    gc.collect()
    junk = [torch.full((1 << 16,), 7, dtype=torch.int32, device="cuda") for _ in range(8)]  # reuse freed blocks
    h = 1.0 / max(N)
    X[:M] = torch.remainder(X[:M] + 0.3 * h * (torch.rand_like(X[:M]) - 0.5), 1.0)
    m.rebin(X)
    fresh = le.Markers(ctx).bin_count(geom, "IB_4", X, torch.tensor([M], dtype=torch.int32, device="cuda"))
    ctx.synchronize()
    assert torch.equal(m.order(), fresh.order())
    del junk


@pytest.mark.parametrize("kernel", ["IB_4", "BSPLINE_4"])
def test_rebin_within_cells_flips_shifted_anchors(le, kernel):
    """Markers that move within their cells change no bucket (the re-binning moves
    nothing) but can change their anchor in the frame shifted by -dz/2, by which the
    spread's candidate stream is split for the side-z / node components (k_cand_write
    SHZ): the re-binning's parities (k_rekey zbits) must send that stream to be rebuilt,
    and a re-binning that changed nothing must keep it."""
    N = (64, 48, 72)
    g = le._lib.load().ibtk_le_min_ghost_width(le.kernel_id(kernel))
    geom = le.Geometry.periodic_unit(list(N), g)
    rng = np.random.default_rng(17)
    M = 30000
    Xn = rng.uniform(0.0, 1.0, (M, 3))
    k = rng.integers(1, N[2] - 1, M)
    Xn[:, 2] = (k - rng.uniform(0.15, 0.25, M)) / N[2]      # z / dz in k - [0.15, 0.25]
    X = torch.from_numpy(Xn).cuda()
    F = torch.from_numpy(rng.standard_normal((M, 3))).cuda()
    Fn = torch.from_numpy(rng.standard_normal((M, 1))).cuda()
    u = _fields(le, geom, rng)
    ctx = le.Context(0)
    m = le.Markers(ctx).bin(geom, kernel, X)

    def node_spread(mk, Xc):
        f = geom.alloc("node", depth=1)
        le.spread(ctx, mk, kernel, "node", geom, f, Fn, Xc)
        ctx.synchronize()
        return f

    _check_same(le, geom, ctx, m, X, F, u, kernel)          # the split stream built
    m.rebin(X)                                               # nothing changed
    _check_same(le, geom, ctx, m, X, F, u, kernel)
    m.rebin(X)                                               # ... again (the parities compared)
    _check_same(le, geom, ctx, m, X, F, u, kernel)
    X2 = X.clone()
    X2[:, 2] += 0.35 / N[2]                                  # z / dz in k + [0.1, 0.2]: the same cells
    m.rebin(X2)
    fr = le.Markers(ctx).bin(geom, kernel, X2)
    assert torch.equal(m.order(), fr.order())
    _check_same(le, geom, ctx, m, X2, F, u, kernel)
    for a, b in zip(node_spread(m, X2), node_spread(fr, X2)):
        assert torch.equal(a, b)
    m.rebin(X2)                                              # nothing changed: the stream stands
    _check_same(le, geom, ctx, m, X2, F, u, kernel)
    m.rebin(X)                                               # and back across
    _check_same(le, geom, ctx, m, X, F, u, kernel)
    for a, b in zip(node_spread(m, X), node_spread(le.Markers(ctx).bin(geom, kernel, X), X)):
        assert torch.equal(a, b)
