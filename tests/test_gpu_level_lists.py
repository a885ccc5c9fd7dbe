"""GPU: a level's index lists in one call (ibtk_le_level_index_lists), against a numpy
restatement of LIndexSetData::cacheLocalIndices (LIndexSetData.cpp:83-169) over every local
patch: the interior lists (markers whose getCellIndex cell, IndexUtilities-inl.h:66-89, lies
in the patch box) and the ghost-box lists (markers and periodic images whose cell lies in
the patch box grown by the ghost width, shifted by +-the domain length), each patch's
entries in its (ghost) box's cell order, x fastest, a cell's markers by index.  Exact:
the same entries in the same order and the same shifts.  Cases: a periodic level with
markers on the domain's faces and corners, a level with patches missing and a
non-periodic dim, a 2-D level, markers crowded into a corner (the ghost-box lists outgrow
the wrapper's first guess: the retry), and the bench's cfg5 lists (bench.level_lists,
torch ops, marker order within a patch) as the same sets.
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


def _cells(X, xlo, xup, dx, dom_lo, dom_hi):
    """getCellIndex in the domain frame (IndexUtilities-inl.h:66-89)."""
    dl, du = X - xlo, X - xup
    lower = np.abs(dl) <= np.abs(du)
    return np.where(lower, dom_lo + np.floor(dl / dx), dom_hi + np.floor(du / dx) + 1).astype(np.int64)


def _expected(X, boxes, dom_lo, dom_hi, dx, xlo, periodic, g):
    nd = X.shape[1]
    xup = xlo + (dom_hi - dom_lo + 1) * dx
    c = _cells(X, xlo, xup, dx, dom_lo, dom_hi)
    ext = dom_hi - dom_lo + 1
    L = ext * dx
    interior, ghost = [], []
    shifts = [np.array(t) for t in np.ndindex(*([3] * nd))]
    for lo, hi in boxes:
        lo, hi = np.array(lo), np.array(hi)
        n = hi - lo + 1
        inside = np.all((c >= lo) & (c <= hi), axis=1)
        s = np.nonzero(inside)[0]
        r = c[s] - lo
        lin = np.zeros(len(s), dtype=np.int64)
        for k in reversed(range(nd)):
            lin = lin * n[k] + r[:, k]
        interior.append(s[np.lexsort((s, lin))])
        ent = []
        for t in shifts:
            sh = t[::-1] - 1  # any order: the entries are sorted below
            if np.any((sh != 0) & ~periodic):
                continue
            ci = c + sh * ext
            ok = np.all((ci >= lo - g) & (ci <= hi + g), axis=1)
            s = np.nonzero(ok)[0]
            r = ci[s] - (lo - g)
            lin = np.zeros(len(s), dtype=np.int64)
            for k in reversed(range(nd)):
                lin = lin * (n[k] + 2 * g) + r[:, k]
            for a, b in zip(lin, s):
                ent.append((a, b, tuple(sh * L)))
        ent.sort(key=lambda e: (e[0], e[1]))
        ghost.append(ent)
    return interior, ghost


def _check(le, ctx, geoms, boxes, dom_lo, dom_hi, dx, xlo, periodic, g, Xn):
    X = torch.from_numpy(Xn).cuda().contiguous()
    (ii, _, oi), (gi, gx, og) = le.level_index_lists(ctx, geoms, dom_lo, dom_hi, X, g,
                                                     periodic=[int(p) for p in periodic])
    exp_i, exp_g = _expected(Xn, boxes, np.array(dom_lo), np.array(dom_hi), np.array(dx), np.array(xlo),
                             np.array(periodic), g)
    ii, gi, gx = ii.cpu().numpy(), gi.cpu().numpy(), gx.cpu().numpy()
    assert oi[-1] == sum(len(e) for e in exp_i) and og[-1] == sum(len(e) for e in exp_g)
    for q in range(len(boxes)):
        np.testing.assert_array_equal(ii[oi[q]:oi[q + 1]], exp_i[q])
        ent = exp_g[q]
        np.testing.assert_array_equal(gi[og[q]:og[q + 1]], np.array([e[1] for e in ent], dtype=np.int64))
        want = np.array([e[2] for e in ent], dtype=np.float64).reshape(-1, Xn.shape[1])
        np.testing.assert_array_equal(gx[og[q]:og[q + 1]], want)
    return (ii, oi), (gi, gx, og)


def _tiles(le, n, P, g, dx, skip=()):
    geoms, boxes = [], []
    nd = len(P)
    for t in np.ndindex(*P[::-1]):
        t = t[::-1]
        if t in skip:
            continue
        lo = [t[k] * n[k] for k in range(nd)]
        hi = [lo[k] + n[k] - 1 for k in range(nd)]
        geoms.append(le.Geometry(lo, hi, g, dx, [lo[k] * dx[k] for k in range(nd)]))
        boxes.append((lo, hi))
    return geoms, boxes


def test_periodic_level_faces_and_corners(le):
    ctx = le.Context(0)
    n, P, g = [12, 10, 8], [4, 3, 5], 3
    N = [n[k] * P[k] for k in range(3)]
    dx = [1.0 / N[0], 0.5 / N[1], 2.0 / N[2]]
    geoms, boxes = _tiles(le, n, P, g, dx)
    rng = np.random.default_rng(3)
    L = np.array([N[k] * dx[k] for k in range(3)])
    Xn = rng.uniform(0.0, 1.0, (20000, 3)) * L
    Xn[:500] = np.round(Xn[:500] / L * 4) / 4 * L        # on faces, edges and corners
    Xn[500:600] = rng.uniform(-0.5, 0.5, (100, 3)) * np.array(dx)  # around the origin corner
    _check(le, ctx, geoms, boxes, [0, 0, 0], [N[0] - 1, N[1] - 1, N[2] - 1], dx, [0.0, 0.0, 0.0],
           [True, True, True], g, Xn)


def test_level_with_missing_patches_and_a_wall(le):
    ctx = le.Context(0)
    n, P, g = [16, 16, 16], [3, 3, 2], 4
    N = [n[k] * P[k] for k in range(3)]
    dx = [1.0 / 48] * 3
    geoms, boxes = _tiles(le, n, P, g, dx, skip={(1, 1, 0), (0, 2, 1), (2, 0, 1)})
    rng = np.random.default_rng(8)
    Xn = rng.uniform(-0.05, 1.05, (15000, 3)) * np.array([N[k] * dx[k] for k in range(3)])  # some outside in z
    _check(le, ctx, geoms, boxes, [0, 0, 0], [N[0] - 1, N[1] - 1, N[2] - 1], dx, [0.0, 0.0, 0.0],
           [True, True, False], g, Xn)


def test_two_dimensional_level(le):
    ctx = le.Context(0)
    n, P, g = [16, 8], [4, 6], 3
    N = [n[k] * P[k] for k in range(2)]
    dx = [1.0 / N[0], 1.0 / N[1]]
    geoms, boxes = _tiles(le, n, P, g, dx)
    rng = np.random.default_rng(2)
    Xn = rng.uniform(0.0, 1.0, (8000, 2))
    _check(le, ctx, geoms, boxes, [0, 0], [N[0] - 1, N[1] - 1], dx, [0.0, 0.0], [True, True], g, Xn)


def test_crowded_corner_grows_the_ghost_lists(le):
    """Every marker within the ghost width of a corner shared by 8 patches and 8 periodic
    images: ~8 ghost-box entries a marker, past the wrapper's first capacity (1.25 per
    marker), so it calls again with the size reported."""
    ctx = le.Context(0)
    n, P, g = [8, 8, 8], [2, 2, 2], 3
    dx = [1.0 / 16] * 3
    geoms, boxes = _tiles(le, n, P, g, dx)
    rng = np.random.default_rng(5)
    Xn = rng.uniform(-2.0, 2.0, (3000, 3)) / 16 % 1.0
    _check(le, ctx, geoms, boxes, [0, 0, 0], [15, 15, 15], dx, [0.0, 0.0, 0.0], [True, True, True], g, Xn)


def test_cfg5_lists_match_the_bench_torch_lists(le):
    """The cfg5 level (512^3 in 8^3 patches, clustered markers, IB_4 ghost width): the device
    lists hold exactly the entries of bench.level_lists (torch ops, marker order within a
    patch), patch by patch."""
    import bench
    from ibamr_amd.slab import Slab
    cfg = bench.CONFIGS["cfg5"]
    N, P, M = cfg["N"], cfg["patches"], cfg["M"]
    n = N // P
    g = le._lib.load().ibtk_le_min_ghost_width(le.kernel_id(cfg["kernel"]))
    ctx = le.Context(0)
    geoms, _ = _tiles(le, [n] * 3, [P] * 3, g, [1.0 / N] * 3)
    X = bench.make_markers("clustered", M // 10, Slab([N, N, N], 1, 0, g), 77, "cuda")
    X = torch.remainder(X, 1.0).contiguous()
    X.masked_fill_(X >= 1.0, 0.0)
    (ii, _, oi), (gi, gx, og) = le.level_index_lists(ctx, geoms, [0, 0, 0], [N - 1] * 3, X, g)
    (ti, _, toi), (tg, tgx, tog) = bench.level_lists(X, N, P, g)
    assert list(oi) == [int(v) for v in toi] and list(og) == [int(v) for v in tog]
    Mx = X.shape[0]

    def canon(idx, xs, off):
        # per patch: entries keyed by (marker, shift) and sorted
        q = torch.repeat_interleave(torch.arange(len(off) - 1, device=idx.device),
                                    torch.tensor(np.diff(off), device=idx.device))
        k = q.long() * Mx + idx.long()
        if xs is not None:
            k = k * 27 + ((xs.round().long() + 1) * torch.tensor([1, 3, 9], device=xs.device)).sum(1)
        return torch.sort(k).values

    assert torch.equal(canon(ii, None, oi), canon(ti.to(ii.device), None, toi))
    assert torch.equal(canon(gi, gx, og), canon(tg, tgx, tog))


def test_marker_order_lists_equal_the_torch_lists(le):
    """order="markers": each patch's entries in marker order -- exactly bench.level_lists'
    lists (torch ops), entry for entry and shift for shift, on a reduced cfg5 level."""
    import bench
    from ibamr_amd.slab import Slab
    N, P, g = 128, 4, 3
    n = N // P
    ctx = le.Context(0)
    geoms, _ = _tiles(le, [n] * 3, [P] * 3, g, [1.0 / N] * 3)
    X = bench.make_markers("clustered", 200000, Slab([N, N, N], 1, 0, g), 5, "cuda")
    X = torch.remainder(X, 1.0).contiguous()
    X.masked_fill_(X >= 1.0, 0.0)
    (ii, _, oi), (gi, gx, og) = le.level_index_lists(ctx, geoms, [0, 0, 0], [N - 1] * 3, X, g, order="markers")
    (ti, _, toi), (tg, tgx, tog) = bench.level_lists(X, N, P, g)
    assert list(oi) == [int(v) for v in toi] and list(og) == [int(v) for v in tog]
    assert torch.equal(ii, ti.to(ii.device))
    assert torch.equal(gi, tg.to(gi.device))
    assert torch.equal(gx, tgx)
    # and the same sets as the cell order
    (ci, _, coi), (cg, cgx, cog) = le.level_index_lists(ctx, geoms, [0, 0, 0], [N - 1] * 3, X, g)
    assert list(coi) == list(oi) and list(cog) == list(og)
    for q in range(len(geoms)):
        a = torch.sort(ii[oi[q]:oi[q + 1]]).values
        b = torch.sort(ci[coi[q]:coi[q + 1]]).values
        assert torch.equal(a, b), q

