"""GPU: local numbering of a patch's markers (ibtk_le_local_numbering, SURVEY.md §8f
row 1) -- LDataManager::computeNodeDistribution (LDataManager.cpp:2839-3027): markers
in the patch box's cells first, in box iteration order (x fastest) and input order
within a cell, then the markers outside the box.  Cells by IndexUtilities::
getCellIndex (IndexUtilities-inl.h:66-89, restated in oracle.get_cell_index).  The
permutation must equal numpy's stable sort of the oracle's keys exactly."""
import numpy as np
import pytest

from oracle import oracle as ora

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


def _expected(X, geom):
    nd = geom.ndim
    c = ora.get_cell_index(X, geom.x_lower, geom.x_upper, geom.dx, geom.ilower, geom.iupper)
    n = [geom.iupper[d] - geom.ilower[d] + 1 for d in range(nd)]
    inside = np.ones(X.shape[0], dtype=bool)
    key = np.zeros(X.shape[0], dtype=np.int64)
    stride = 1
    for d in range(nd):
        inside &= (c[:, d] >= geom.ilower[d]) & (c[:, d] <= geom.iupper[d])
        key += (c[:, d] - geom.ilower[d]) * stride
        stride *= n[d]
    key[~inside] = stride
    return np.argsort(key, kind="stable"), int(inside.sum())


@pytest.mark.parametrize("ndim", [2, 3])
@pytest.mark.parametrize("M", [0, 1, 1000, 200_003])
def test_local_numbering_matches_stable_cell_sort(le, ctx, ndim, M):
    N, ilo = [40, 24, 16], [2, -3, 0]
    geom = le.Geometry(ilo[:ndim], [ilo[d] + N[d] - 1 for d in range(ndim)], 2, [0.05] * ndim,
                       [0.1, -0.15, 0.0][:ndim])
    rng = np.random.default_rng(M + ndim)
    lo = np.array(geom.x_lower)
    hi = np.array(geom.x_upper)
    # a tenth outside the patch, some exactly on cell faces (getCellIndex's corner rule)
    X = rng.uniform(lo - 0.1 * (hi - lo), hi + 0.1 * (hi - lo), (M, ndim))
    if M:
        k = max(1, M // 20)
        X[:k] = lo + np.round((X[:k] - lo) / 0.05) * 0.05
    order, nin = le.local_numbering(ctx, geom, torch.from_numpy(X).cuda())
    exp, exp_in = _expected(X, geom)
    assert nin == exp_in
    assert np.array_equal(order.cpu().numpy(), exp)


def _level(le, P, n, g, order_perm=None, subset=None, dx=None, z_extra=(0, 0)):
    """Patches of n^3 tiling a periodic P^3 domain (optionally a subset, in a given
    PatchLevel order); returns (geoms, boxes, dom_lo, dom_hi, dx)."""
    N = P * n
    dx = dx or 1.0 / N
    tiles = [(i, j, k) for k in range(P) for j in range(P) for i in range(P)]
    if subset is not None:
        tiles = [t for t in tiles if subset(t)]
    if order_perm is not None:
        tiles = [tiles[i] for i in order_perm(len(tiles))]
    geoms, boxes = [], []
    for t in tiles:
        lo = [t[d] * n for d in range(3)]
        hi = [lo[d] + n - 1 for d in range(3)]
        geoms.append(le.Geometry(lo, hi, g, [dx] * 3, [lo[d] * dx for d in range(3)]))
        boxes.append((lo, hi))
    return geoms, boxes, [0, 0, 0], [N - 1] * 3, dx


@pytest.mark.parametrize("case", ["all_local", "half_level", "slab_with_ghosts"])
def test_level_node_distribution_matches_oracle(le, ctx, case):
    """LDataManager::computeNodeDistribution over a level's local patches (ibtk_le_level_
    node_distribution) entry by entry against the oracle's loop restatement
    (LDataManager.cpp:2874-2947): a clustered level of 4^3 patches of 6^3 cells in a
    shuffled PatchLevel order, with repeated Lagrangian indices; half the level local
    (the others' markers near the boundary are nonlocal ghost nodes, periodic images
    included); a z-slab rank holding its own markers plus the neighbours' ghost markers."""
    P, n, g = 4, 6, 2
    rng = np.random.default_rng(7)
    perm = lambda k: list(rng.permutation(k))
    if case == "all_local":
        geoms, boxes, dlo, dhi, dx = _level(le, P, n, g, order_perm=perm)
    elif case == "half_level":
        geoms, boxes, dlo, dhi, dx = _level(le, P, n, g, order_perm=perm, subset=lambda t: (t[0] + t[2]) % 2 == 0)
    else:
        geoms, boxes, dlo, dhi, dx = _level(le, P, n, g, subset=lambda t: t[2] == 1)
    M = 3000
    X = rng.uniform(0, 1, (M, 3))
    X[:1000, 2] = 0.40 + (X[:1000, 2] - 0.5) / (P * n)           # a sheet one cell thick
    X[1000:1500, :2] = 0.3 + 0.02 * rng.standard_normal((500, 2))  # a bundle along z
    X = np.mod(X, 1.0)
    lag = rng.permutation(M).astype(np.int32)
    lag[2000:2030] = lag[:30]                                      # repeated Lagrangian indices
    X[2000:2030] = X[:30]
    Xd = torch.from_numpy(X).cuda()
    order, nl, nn = le.level_node_distribution(ctx, geoms, dlo, dhi, Xd, g, lag=torch.from_numpy(lag).cuda())
    eo, enl, enn = ora.level_node_distribution(X, lag, boxes, dlo, dhi, [0.0] * 3, [dx] * 3, g)
    assert (nl, nn) == (enl, enn)
    if case != "all_local":
        assert nn > 0
    assert np.array_equal(order.cpu().numpy(), eo)
    # the LData reorder: row i of the new arrays is the old row order[i]
    F = torch.from_numpy(rng.standard_normal((M, 3))).cuda()
    Xn, Fn = le.ldata_reorder(ctx, order, Xd, F)
    assert torch.equal(Xn, Xd[order.long()]) and torch.equal(Fn, F[order.long()])


def test_wrap_positions_matches_reference_loops(le, ctx):
    """beginDataRedistribution's wrap (LDataManager.cpp:1385-1399) on the device, bit for
    bit against the reference's loops restated in Python: while X < lower add the length,
    while X >= upper subtract it (periodic dims), then clamp into [lower, upper - eps]."""
    rng = np.random.default_rng(5)
    lo, hi = [0.0, -0.5, 0.25], [1.0, 0.75, 2.0]
    X = rng.uniform(-3.0, 4.0, (5000, 3))
    X[:10] = [[1.0, 0.75, 2.0]] * 10             # exactly on the upper faces
    X[10:20] = [[-1e-17, -0.5, 0.25]] * 10        # just below / on the lower faces
    periodic = [1, 0, 1]
    exp = X.copy()
    eps = np.finfo(np.float64).eps
    for i in range(X.shape[0]):
        for d in range(3):
            x = exp[i, d]
            if periodic[d]:
                Ld = hi[d] - lo[d]
                while x < lo[d]:
                    x += Ld
                while x >= hi[d]:
                    x -= Ld
            x = max(x, lo[d])
            x = min(x, hi[d] - eps)
            exp[i, d] = x
    Xd = torch.from_numpy(X.copy()).cuda()
    le.wrap_positions(ctx, Xd, lo, hi, periodic=periodic)
    assert np.array_equal(Xd.cpu().numpy(), exp)
    # a NaN coordinate stays NaN in a non-periodic dim (std::max / std::min keep it,
    # LDataManager.cpp:1398-1399; fmax / fmin would clamp it to the lower face)
    Xn = torch.tensor([[0.5, float("nan"), 1.0], [0.5, 0.1, 1.0]], dtype=torch.float64, device="cuda")
    le.wrap_positions(ctx, Xn, lo, hi, periodic=periodic)
    out = Xn.cpu().numpy()
    assert np.isnan(out[0, 1]) and out[1, 1] == 0.1 and out[0, 0] == 0.5
