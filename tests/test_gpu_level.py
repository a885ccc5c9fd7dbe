"""GPU: a level of patches in one launch per sweep (ibtk_le_level_*), against the
per-patch calls and the oracle run patch by patch -- LDataManager::interp /
spread's patch loop (LDataManager.cpp:625-660, 763-807; SURVEY.md 8(d) cfg5's
multi-patch finest level).

Each patch has its own ghosted side arrays, filled from one periodic field;
interp takes the patch's interior list (markers whose cell is in the patch
box), spread the patch's ghost-box list (the markers and periodic images whose
cell is in the ghost box, as the index data's ghost box holds them), so every
patch's interior is complete without a grid reduction.
Interp must equal the per-patch result bit for bit, spread within 1e-12 of the
oracle on each patch (the sweep sums each point in a fixed order), and both
bit-stable run to run.
"""
import itertools

import numpy as np
import pytest

from oracle import oracle as ora

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu
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


def _patches(le, N, P, g):
    n = N // P
    dx = 1.0 / N
    geoms = []
    for k, j, i in itertools.product(range(P), repeat=3):
        lo = [i * n, j * n, k * n]
        geoms.append(le.Geometry(lo, [l + n - 1 for l in lo], g, [dx] * 3, [l * dx for l in lo]))
    return geoms


def _fill(geom, G, N):
    """side arrays of the patch, values of the periodic field G[c] (z, y, x) at every point"""
    out = []
    for c in range(3):
        shp = geom.array_shape("side", c)
        zz = np.arange(shp[0]) + geom.ilower[2] - geom.gcw[2]
        yy = np.arange(shp[1]) + geom.ilower[1] - geom.gcw[1]
        xx = np.arange(shp[2]) + geom.ilower[0] - geom.gcw[0]
        out.append(np.ascontiguousarray(G[c][np.ix_(zz % N, yy % N, xx % N)]))
    return out


def _lists(geom, X, N, g):
    dx = 1.0 / N
    c = np.floor(X / dx).astype(np.int64)
    lo, hi = np.array(geom.ilower), np.array(geom.iupper)
    inside = np.all((c >= lo) & (c <= hi), axis=1)
    interior = np.nonzero(inside)[0].astype(np.int32)
    idx, xs = [], []
    for s in itertools.product((-1, 0, 1), repeat=3):
        ci = c + np.array(s) * N
        ok = np.all((ci >= lo - g) & (ci <= hi + g), axis=1)
        sel = np.nonzero(ok)[0]
        idx.append(sel)
        xs.append(np.tile(np.array(s, np.float64), (sel.size, 1)))
    idx = np.concatenate(idx).astype(np.int32)
    xs = np.concatenate(xs)
    o = np.argsort(idx, kind="stable")
    return interior, idx[o], xs[o]


@pytest.mark.parametrize("kernel,P,clustered", [("IB_4", 2, False), ("IB_6", 2, False), ("IB_4", 4, True),
                                                ("BSPLINE_4", 2, True)])
def test_level_matches_patch_by_patch(le, ctx, kernel, P, clustered):
    N = 64 if P == 4 else 48
    g = ora.min_ghost_width(kernel)
    geoms = _patches(le, N, P, g)
    rng = np.random.default_rng(3 + P)
    M = 40_000
    X = rng.uniform(0, 1, (M, 3))
    if clustered:  # a sheet one cell thick and a fibre bundle along z
        X[: M // 2, 2] = 0.5 + (rng.uniform(0, 1, M // 2) - 0.5) / N
        r, t = 0.05 * np.sqrt(rng.uniform(0, 1, M // 4)), 2 * np.pi * rng.uniform(0, 1, M // 4)
        X[M // 2: M // 2 + M // 4, 0] = 0.3 + r * np.cos(t)
        X[M // 2: M // 2 + M // 4, 1] = 0.6 + r * np.sin(t)
    F = rng.uniform(-1, 1, (M, 3))
    G = [rng.uniform(-1, 1, (N, N, N)) for _ in range(3)]
    Xd, Fd = torch.from_numpy(X).cuda(), torch.from_numpy(F).cuda()
    lists_i, lists_s, host = [], [], []
    for geom in geoms:
        interior, idx, xs = _lists(geom, X, N, g)
        host.append((interior, idx, xs))
        lists_i.append((torch.from_numpy(interior).cuda(), None))
        lists_s.append((torch.from_numpy(idx).cuda(), torch.from_numpy(xs).cuda()))
    u = [[torch.from_numpy(a).cuda() for a in _fill(geom, G, N)] for geom in geoms]
    # interp: one launch over the level
    lvl_i = le.Level(ctx, geoms, kernel, Xd, lists_i)
    U = torch.full((M, 3), np.nan, dtype=torch.float64, device="cuda")
    lvl_i.interp("side", u, U, Xd)
    # spread: one launch, twice (bit stability)
    lvl_s = le.Level(ctx, geoms, kernel, Xd, lists_s)
    outs = []
    for rep in range(2):
        f = [[torch.zeros_like(a) for a in per] for per in u]
        lvl_s.spread("side", f, Fd, Xd)
        outs.append(f)
    # one binning for both sweeps: the ghost-box binning told the interior lists
    # (ibtk_le_level_select_interior) interpolates bit for bit as the interior binning
    offs = [0]
    for l in lists_i:
        offs.append(offs[-1] + l[0].numel())
    lvl_s.select_interior(M, torch.cat([l[0] for l in lists_i]), offs)
    U2 = torch.full((M, 3), np.nan, dtype=torch.float64, device="cuda")
    lvl_s.interp("side", u, U2, Xd)
    ctx.synchronize()
    assert torch.equal(U2, U), "interp on the selected interior entries of the ghost-box binning"
    Ug = U.cpu().numpy()
    assert not np.isnan(Ug).any(), "every marker is interior to exactly one patch"
    for q, geom in enumerate(geoms):
        interior, idx, xs = host[q]
        # the single-patch device call on the same list: interp bit for bit
        m = le.Markers(ctx).bin(geom, kernel, Xd, torch.from_numpy(interior).cuda())
        U1 = torch.zeros((M, 3), dtype=torch.float64, device="cuda")
        le.interp(ctx, m, kernel, "side", geom, u[q], U1, Xd)
        ctx.synchronize()
        assert np.array_equal(Ug[interior], U1.cpu().numpy()[interior]), f"patch {q} interp"
        # and the level interp directly against the oracle on the patch's interior list:
        # bit for bit (the Fortran's order and roundings)
        Qo = np.zeros((M, 3))
        ora.side_interp(kernel, geom.dx, geom.x_lower, geom.ilower, geom.iupper, geom.gcw,
                        [a.cpu().numpy() for a in u[q]], interior, np.zeros((interior.size, 3)), X, Qo)
        assert np.array_equal(Ug[interior], Qo[interior]), f"patch {q} level interp vs oracle"
        # the oracle on the patch's ghost-box list
        uo = [np.zeros(tuple(a.shape)) for a in u[q]]
        ora.side_spread(kernel, geom.dx, geom.x_lower, geom.ilower, geom.iupper, geom.gcw, uo, idx, xs, X, F)
        for a in range(3):
            got = outs[0][q][a].cpu().numpy()
            assert np.array_equal(got, outs[1][q][a].cpu().numpy()), f"patch {q} comp {a} not bit-stable"
            err = np.abs(got - uo[a]).max() / max(np.abs(uo[a]).max(), 1e-300)
            assert err <= SPREAD_TOL, f"patch {q} comp {a} spread rel err {err:.2e}"
    # the level's interiors are the periodic spread: conservation over unique points
    h3 = geoms[0].dx[0] ** 3
    for a in range(3):
        tot = 0.0
        for q, geom in enumerate(geoms):
            n = geom.iupper[0] - geom.ilower[0] + 1
            tot += outs[0][q][a][g:g + n, g:g + n, g:g + n].sum().item()
        assert abs(tot * h3 - F[:, a].sum()) <= 1e-10 * np.abs(F[:, a]).sum()


def test_level_rejects_single_patch_calls(le, ctx):
    from ibamr_amd._lib import IBTKLEError
    geoms = _patches(le, 32, 2, 3)
    X = torch.rand((100, 3), dtype=torch.float64, device="cuda")
    lvl = le.Level(ctx, geoms, "IB_4", X, [None] * len(geoms))
    u = geoms[0].alloc("side")
    Q = torch.zeros((100, 3), dtype=torch.float64, device="cuda")
    with pytest.raises(IBTKLEError):
        le.interp(ctx, lvl.markers, "IB_4", "side", geoms[0], u, Q, X)


@pytest.mark.parametrize("P", [2, 4])
def test_level_fill_ghosts(le, ctx, P):
    """Every ghost point of every patch takes the value of the patch owning it
    (periodic wrap), the schedule fill before interp (LDataManager.cpp:748-751)."""
    N, g = 32, 3
    geoms = _patches(le, N, P, g)
    rng = np.random.default_rng(P)
    G = [rng.uniform(-1, 1, (N, N, N)) for _ in range(3)]
    want = [_fill(geom, G, N) for geom in geoms]
    n = N // P
    arrays = []
    for geom, w in zip(geoms, want):
        per = []
        for a in range(3):
            t = torch.full(w[a].shape, np.nan, dtype=torch.float64, device="cuda")
            t[g:g + n, g:g + n, g:g + n] = torch.from_numpy(w[a][g:g + n, g:g + n, g:g + n]).cuda()
            per.append(t)
        arrays.append(per)
    X = torch.rand((10, 3), dtype=torch.float64, device="cuda")
    lvl = le.Level(ctx, geoms, "IB_4", X, [None] * len(geoms))
    lvl.fill_ghosts("side", arrays)
    ctx.synchronize()
    for q in range(len(geoms)):
        for a in range(3):
            assert np.array_equal(arrays[q][a].cpu().numpy(), want[q][a]), f"patch {q} comp {a}"


@pytest.mark.parametrize("centering,depth", [("side", 1), ("cell", 1), ("cell", 2), ("node", 1)])
def test_level_zero(le, ctx, centering, depth):
    """ibtk_le_level_zero: every element of every patch array (ghosts included)
    := 0, and nothing beyond the arrays (LDataManager.cpp:596's setToScalar)."""
    geoms = _patches(le, 18, 2, 3)  # 9^3 patches: 15^3 cell arrays, an odd count
    per = 3 if centering == "side" else 1
    arrays, guards = [], []
    for geom in geoms:
        row = []
        for a in range(per):
            shp = geom.array_shape(centering, a, depth)
            n = int(np.prod(shp))
            buf = torch.full((n + 2,), np.nan, dtype=torch.float64, device="cuda")
            row.append(buf[1:n + 1].view(shp))  # 8-byte aligned views: the scalar path
            guards.append(buf)
        arrays.append(row)
    X = torch.rand((10, 3), dtype=torch.float64, device="cuda")
    lvl = le.Level(ctx, geoms, "IB_4", X, [None] * len(geoms))
    lvl.zero(centering, arrays, q_depth=depth)
    ctx.synchronize()
    for buf in guards:
        b = buf.cpu().numpy()
        assert np.isnan(b[0]) and np.isnan(b[-1]), "wrote outside the array"
        assert not b[1:-1].any() and not np.isnan(b[1:-1]).any()
    # 16-byte aligned arrays (the vector path)
    f = [geom.alloc(centering, depth=depth, fill=float("nan")) for geom in geoms]
    lvl.zero(centering, f, q_depth=depth)
    ctx.synchronize()
    assert all(not t.cpu().numpy().any() for row in f for t in row)


def test_level_select_interior_rejects_foreign_entries(le, ctx):
    """An interior list naming a marker its patch's binned list does not hold raises
    device flag 4 at the next synchronize."""
    g = ora.min_ghost_width("IB_4")
    N, P = 32, 2
    n = N // P
    dx = 1.0 / N
    geoms = []
    for k in range(P):
        for j in range(P):
            for i in range(P):
                lo = [i * n, j * n, k * n]
                geoms.append(le.Geometry(lo, [v + n - 1 for v in lo], g, [dx] * 3, [v * dx for v in lo]))
    X = torch.full((4, 3), 0.1, dtype=torch.float64, device="cuda")  # all in patch 0
    lists = [(torch.arange(4, dtype=torch.int32, device="cuda"), None)] + \
            [(torch.zeros(0, dtype=torch.int32, device="cuda"), None)] * (len(geoms) - 1)
    lvl = le.Level(ctx, geoms, "IB_4", X, lists)
    offs = [0] + [4] * len(geoms)           # patch 0's interior list: markers 0..3 -- fine
    lvl.select_interior(4, torch.arange(4, dtype=torch.int32, device="cuda"), offs)
    ctx.synchronize()
    offs = [0, 0, 4] + [4] * (len(geoms) - 2)  # patch 1 claims them: not in its list
    lvl.select_interior(4, torch.arange(4, dtype=torch.int32, device="cuda"), offs)
    with pytest.raises(RuntimeError, match="flag 4"):
        ctx.synchronize()
    # an interior list naming a marker past n_markers (and a binned list beyond it):
    # flagged, never dereferenced
    offs = [0] + [4] * len(geoms)
    lvl.select_interior(4, torch.tensor([0, 1, 2, 1 << 20], dtype=torch.int32, device="cuda"), offs)
    with pytest.raises(RuntimeError, match="flag 4"):
        ctx.synchronize()
    lvl.select_interior(2, torch.tensor([0, 1], dtype=torch.int32, device="cuda"), [0] + [2] * len(geoms))
    with pytest.raises(RuntimeError, match="flag 4"):
        ctx.synchronize()


@pytest.mark.parametrize("kernel,clustered", [("IB_4", True), ("IB_6", False)])
def test_level_zero_spread(le, ctx, kernel, clustered):
    """ibtk_le_level_zero_spread (LDataManager::spread's setToScalar(f, 0, false) and
    patch loop in one launch) equals ibtk_le_level_zero then ibtk_le_level_spread bit
    for bit, on arrays that start as NaN -- every point of every array is written,
    including the patches and columns no marker reaches."""
    N, P = 48, 2
    g = ora.min_ghost_width(kernel)
    geoms = _patches(le, N, P, g)
    rng = np.random.default_rng(11)
    M = 20_000
    X = rng.uniform(0, 1, (M, 3))
    if clustered:  # a sheet inside the lower patches only: the upper ones get no marker
        X[:, 2] = 0.2 + (rng.uniform(0, 1, M) - 0.5) / N
    F = rng.uniform(-1, 1, (M, 3))
    Xd, Fd = torch.from_numpy(X).cuda(), torch.from_numpy(F).cuda()
    lists = []
    for geom in geoms:
        _, idx, xs = _lists(geom, X, N, g)
        lists.append((torch.from_numpy(idx).cuda(), torch.from_numpy(xs).cuda()))
    lvl = le.Level(ctx, geoms, kernel, Xd, lists)
    want = [geom.alloc("side", fill=float("nan")) for geom in geoms]
    lvl.zero("side", want)
    lvl.spread("side", want, Fd, Xd)
    got = [geom.alloc("side", fill=float("nan")) for geom in geoms]
    lvl.zero_spread("side", got, Fd, Xd)
    ctx.synchronize()
    for q in range(len(geoms)):
        for a in range(3):
            w, o = want[q][a].cpu().numpy(), got[q][a].cpu().numpy()
            assert not np.isnan(o).any(), f"patch {q} comp {a}: points not written"
            assert np.array_equal(w, o), f"patch {q} comp {a}"
    # an empty level binning: the zeroing alone
    empty = le.Level(ctx, geoms, kernel, Xd, [(torch.zeros(0, dtype=torch.int32, device="cuda"),
                                                torch.zeros((0, 3), dtype=torch.float64, device="cuda"))] * len(geoms))
    f = [geom.alloc("side", fill=float("nan")) for geom in geoms]
    empty.zero_spread("side", f, Fd, Xd)
    ctx.synchronize()
    assert all(not t.cpu().numpy().any() and not np.isnan(t.cpu().numpy()).any() for row in f for t in row)


@pytest.mark.parametrize("kernel,P,centering,periodic,window", [
    ("IB_4", 2, "side", (1, 1, 1), True), ("IB_4", 4, "side", (1, 1, 1), True),
    ("IB_6", 2, "side", (1, 1, 1), True), ("PIECEWISE_CUBIC", 2, "side", (1, 1, 1), True),
    ("IB_4", 2, "side", (1, 0, 1), True), ("IB_4", 4, "side", (0, 1, 0), True),
    ("IB_4", 2, "cell", (1, 1, 1), True), ("BSPLINE_4", 2, "side", (1, 1, 0), True),
    ("IB_4", 2, "side", (1, 1, 1), "scattered"), ("IB_4", 2, "side", (1, 1, 1), "far"),
    ("IB_4", 4, "side", (1, 1, 1), "small")])
def test_level_fill_interp(le, ctx, kernel, P, centering, periodic, window):
    """ibtk_le_level_fill_interp equals ibtk_le_level_fill_ghosts then ibtk_le_level_interp,
    Q bit for bit, and writes no array point: the fused sweep reads a ghost point in the
    neighbour patch the fill copies it from.  Ghost points that have a neighbour are NaN in the
    fused call's arrays (never read); across non-periodic faces, where the fill copies nothing,
    both calls read the same values.  window "scattered": an allocation per array (still within
one 2-GB window: fused, through the offset table); "far": patch 0's arrays more than 2 GB
from the others (the two calls)."""
    N = 96 if P == 2 else 192  # patches of 48 cells: the fused form
    if window == "small":  # 12-cell patches: the two calls
        N = 48
    g = ora.min_ghost_width(kernel)
    geoms = _patches(le, N, P, g)
    rng = np.random.default_rng(7 + P)
    M = 30_000
    X = rng.uniform(0, 1, (M, 3))
    Xd = torch.from_numpy(X).cuda()
    lists_i = [(torch.from_numpy(_lists(geom, X, N, g)[0]).cuda(), None) for geom in geoms]
    lvl = le.Level(ctx, geoms, kernel, Xd, lists_i)
    ncomp = 3 if centering == "side" else 1
    spacer = None
    if window is True or window == "small":
        a_arr = le.alloc_level(geoms, centering)
        b_arr = le.alloc_level(geoms, centering)
    elif window == "scattered":
        a_arr = [geom.alloc(centering) for geom in geoms]
        b_arr = [geom.alloc(centering) for geom in geoms]
    else:
        a_arr, b_arr = [geoms[0].alloc(centering)], [geoms[0].alloc(centering)]
        spacer = torch.empty(int(2.2 * 2**30) // 8, dtype=torch.float64, device="cuda")
        a_arr += [geom.alloc(centering) for geom in geoms[1:]]
        b_arr += [geom.alloc(centering) for geom in geoms[1:]]
    n = N // P
    for q, geom in enumerate(geoms):
        tile = [(geom.ilower[d] // n) for d in range(3)]
        for a in range(ncomp):
            v = rng.uniform(-1, 1, tuple(a_arr[q][a].shape))
            a_arr[q][a].copy_(torch.from_numpy(v))
            # the fused call's ghosts: NaN wherever a neighbour patch supplies them
            w = v.copy()
            shp = v.shape[-3:]  # (z, y, x) (cell data: a leading depth)
            idx = [np.arange(shp[2 - d]) + geom.ilower[d] - g for d in range(3)]  # global index per dim (x, y, z)
            dirs = [np.where(idx[d] < geom.ilower[d], -1, np.where(idx[d] >= geom.ilower[d] + n, 1, 0)) for d in range(3)]
            ok = [np.where(dirs[d] == 0, True, bool(periodic[d]) |
                           ((tile[d] + dirs[d] >= 0) & (tile[d] + dirs[d] < P))) for d in range(3)]
            ghost = (dirs[2][:, None, None] != 0) | (dirs[1][None, :, None] != 0) | (dirs[0][None, None, :] != 0)
            supplied = ok[2][:, None, None] & ok[1][None, :, None] & ok[0][None, None, :]
            w[..., ghost & supplied] = np.nan
            b_arr[q][a].copy_(torch.from_numpy(w))
    b_before = [[t.clone() for t in per] for per in b_arr]
    Qd = 3 if centering == "side" else 1
    Qa = torch.full((M, Qd), np.nan, dtype=torch.float64, device="cuda")
    Qb = torch.full_like(Qa, np.nan)
    lvl.fill_ghosts(centering, a_arr, periodic=list(periodic))
    lvl.interp(centering, a_arr, Qa, Xd, Q_depth=Qd)
    lvl.fill_interp(centering, b_arr, Qb, Xd, Q_depth=Qd, periodic=list(periodic))
    ctx.synchronize()
    qa, qb = Qa.cpu().numpy(), Qb.cpu().numpy()
    assert not np.isnan(qb).any(), "a NaN ghost (one a neighbour supplies) was read"
    assert np.array_equal(qa, qb), f"max diff {np.abs(qa - qb).max()}"
    if window not in ("far", "small"):  # (the two calls' fill writes the ghosts)
        for per0, per1 in zip(b_before, b_arr):
            for t0, t1 in zip(per0, per1):
                assert torch.equal(torch.nan_to_num(t0, nan=7.0), torch.nan_to_num(t1, nan=7.0)), \
                    "an array point was written"
    del spacer


def test_level_select_interior_cache(le, ctx):
    """A repeated selection of the same interior lists after a re-binning
    (ibtk_le_level_select_interior's cache): kept when no marker changed bucket, made
    again when some did -- the interp equal bit for bit to a fresh level's."""
    kernel, N, P = "IB_4", 32, 2
    g = ora.min_ghost_width(kernel)
    geoms = _patches(le, N, P, g)
    rng = np.random.default_rng(11)
    M = 6000
    X = rng.uniform(0.05, 0.95, (M, 3))
    G = [rng.uniform(-1, 1, (N, N, N)) for _ in range(3)]
    u = [[torch.from_numpy(a).cuda() for a in _fill(geom, G, N)] for geom in geoms]
    lists_i, lists_s = [], []
    for geom in geoms:
        interior, idx, xs = _lists(geom, X, N, g)
        lists_i.append(torch.from_numpy(interior).cuda())
        lists_s.append((torch.from_numpy(idx).cuda(), torch.from_numpy(xs).cuda()))
    offs = [0]
    for l in lists_i:
        offs.append(offs[-1] + l.numel())
    ii = torch.cat(lists_i)

    def interp(level, Xq):
        U = torch.full((M, 3), np.nan, dtype=torch.float64, device="cuda")
        level.interp("side", u, U, Xq)
        return U

    Xd = torch.from_numpy(X).cuda()
    lvl = le.Level(ctx, geoms, kernel, Xd, lists_s)
    lvl.select_interior(M, ii, offs)
    U0 = interp(lvl, Xd)
    assert not torch.isnan(U0).any()
    lvl.rebin(Xd)  # nothing moved: the selection stands
    lvl.select_interior(M, ii, offs)
    assert torch.equal(interp(lvl, Xd), U0)
    # moved a fraction of a cell (within the lists' ghost slack): many change bucket
    X1d = torch.from_numpy(X + rng.uniform(-0.3, 0.3, X.shape) / N).cuda()
    lvl.rebin(X1d)
    lvl.select_interior(M, ii, offs)
    U1 = interp(lvl, X1d)
    ref = le.Level(ctx, geoms, kernel, X1d, lists_s)
    ref.select_interior(M, ii.clone(), offs)
    assert torch.equal(U1, interp(ref, X1d))
    assert not torch.equal(U1, U0)
    lvl.rebin(X1d)  # and nothing moved again
    lvl.select_interior(M, ii, offs)
    assert torch.equal(interp(lvl, X1d), U1)
    ctx.synchronize()
