"""GPU: the index bookkeeping of LDataManager / LIndexSetData, entry by entry
against the oracle.

* ibtk_le_index_set_list -- LIndexSetData::cacheLocalIndices (LIndexSetData.cpp:
  83-169): the ghost box's cells in iteration order (x fastest), each cell's
  markers by Lagrangian index (LDataManager.cpp:1487-1493), with the periodic
  shift of the image's cell; the all / interior / ghost lists.  Indices and
  Xshift must be equal bit for bit.
* ibtk_le_node_distribution -- LDataManager::computeNodeDistribution (LDataManager.
  cpp:2874-2947): local nodes in (cell, Lagrangian index) order, uniqued, then the
  ghost cells' nodes.
* Both are functions of the markers, not of their storage order: after a
  reshuffle of the local storage (what slab.migrate(cell_order=False) does to
  arrivals), the Lagrangian-index sequences are identical.
"""
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


def _case(le, ndim, M, seed, dup_lag=False):
    N = [24, 20, 16][:ndim]
    ilo = [0] * ndim
    geom = le.Geometry.periodic_unit(N, 3)
    rng = np.random.default_rng(seed)
    X = rng.uniform(0.0, 1.0, (M, ndim))
    # some exactly on cell faces (getCellIndex's lower/upper corner rule), the
    # domain's lower face included (positions are wrapped into [0, 1))
    k = max(1, M // 10)
    X[:k] = np.floor(X[:k] * np.array(N)) / np.array(N)
    lag = rng.permutation(M).astype(np.int32) * 3 + 7
    if dup_lag and M > 10:
        lag[M // 2:M // 2 + 5] = lag[:5]  # repeated Lagrangian indices (a marker registered twice)
    return geom, X, lag


@pytest.mark.parametrize("ndim", [2, 3])
@pytest.mark.parametrize("which", ["all", "interior", "ghost"])
@pytest.mark.parametrize("with_lag", [False, True])
def test_index_set_list_matches_oracle(le, ctx, ndim, which, with_lag):
    geom, X, lag = _case(le, ndim, 3000, 5 + ndim)
    g = 3
    Xd = torch.from_numpy(X).cuda()
    lg = torch.from_numpy(lag).cuda() if with_lag else None
    idx, xs = le.index_set_list(ctx, geom, Xd, g, lag=lg, which=which)
    ei, ex, _ = ora.periodic_index_list(X, geom.x_lower, geom.x_upper, geom.dx, geom.ilower, geom.iupper, g,
                                        lag=lag if with_lag else None, which=which)
    assert np.array_equal(idx.cpu().numpy(), ei)
    assert np.array_equal(xs.cpu().numpy(), ex)


@pytest.mark.parametrize("ndim", [2, 3])
def test_index_set_list_uniques_repeated_lagrangian_indices(le, ctx, ndim):
    """Markers sharing a cell and a Lagrangian index are one LNode of the cell's set
    (LDataManager.cpp:1487-1493): the device list drops the later ones as the oracle
    does (lowest marker index kept), in every cell incl. the images'."""
    geom, X, lag = _case(le, ndim, 3000, 21 + ndim, dup_lag=True)
    X[1500:1505] = X[:5]  # the repeated Lagrangian indices on the same positions: same cells
    g = 3
    Xd = torch.from_numpy(X).cuda()
    idx, xs = le.index_set_list(ctx, geom, Xd, g, lag=torch.from_numpy(lag).cuda(), which="all")
    ei, ex, _ = ora.periodic_index_list(X, geom.x_lower, geom.x_upper, geom.dx, geom.ilower, geom.iupper, g,
                                        lag=lag, which="all")
    full, _, _ = ora.periodic_index_list(X, geom.x_lower, geom.x_upper, geom.dx, geom.ilower, geom.iupper, g,
                                         which="all")
    assert ei.size < full.size  # the duplicates were there to drop
    assert np.array_equal(idx.cpu().numpy(), ei) and np.array_equal(xs.cpu().numpy(), ex)


BOXES3 = [((-3, -3, -3), (26, 22, 18)),   # the ghost box: the all list
          ((0, 0, 0), (23, 19, 15)),      # the patch box: the interior list
          ((-2, 4, -3), (5, 19, 2)),      # reaches below the patch in x and z
          ((20, -3, 10), (26, 3, 18)),    # above in x and z, below in y
          ((7, 7, 7), (7, 7, 7))]         # one cell


@pytest.mark.parametrize("with_lag", [False, True])
@pytest.mark.parametrize("box", BOXES3, ids=lambda b: f"{b[0]}-{b[1]}")
def test_index_set_box_list_matches_build_local_indices(le, ctx, box, with_lag):
    """LEInteractor::buildLocalIndices' box branch (LEInteractor.cpp:3070-3106) on the
    device (ibtk_le_index_set_box_list, and ibtk_le_list_in_box over the cached
    all-nodes list with its cells) against the oracle's cell-walk restatement, entry by
    entry: indices, periodic shifts and cells."""
    geom, X, lag = _case(le, 3, 4000, 31, dup_lag=with_lag)
    g = 3
    Xd = torch.from_numpy(X).cuda()
    lg = torch.from_numpy(lag).cuda() if with_lag else None
    idx, xs, cells = le.index_set_box_list(ctx, geom, Xd, g, box[0], box[1], lag=lg)
    sets = ora.lnode_set_data(X, geom.x_lower, geom.x_upper, geom.dx, geom.ilower, geom.iupper, g,
                              lag=lag if with_lag else None)
    ei, ex, ec = ora.build_local_indices(sets, geom.dx, geom.ilower, geom.iupper, g, box)
    assert np.array_equal(idx.cpu().numpy(), ei)
    assert np.array_equal(xs.cpu().numpy(), ex)
    assert np.array_equal(cells.cpu().numpy(), ec)
    # the facade's path: the all-nodes list with its cells, filtered by the box
    ai, ax, ac = le.index_set_box_list(ctx, geom, Xd, g, BOXES3[0][0], BOXES3[0][1], lag=lg)
    fi, fx = le.list_in_box(ctx, ac, ai, ax, box[0], box[1])
    assert np.array_equal(fi.cpu().numpy(), ei) and np.array_equal(fx.cpu().numpy(), ex)


def test_periodic_index_list_is_the_all_list(le, ctx):
    geom, X, lag = _case(le, 3, 2000, 11)
    Xd = torch.from_numpy(X).cuda()
    a = le.periodic_index_list(ctx, geom, Xd, 3)
    b = le.index_set_list(ctx, geom, Xd, 3)
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])


@pytest.mark.parametrize("ndim", [2, 3])
@pytest.mark.parametrize("M", [0, 1, 5000, 120_001])
@pytest.mark.parametrize("ghost", [0, 2])
def test_node_distribution_matches_oracle(le, ctx, ndim, M, ghost):
    N, ilo = [40, 24, 16], [2, -3, 0]
    geom = le.Geometry(ilo[:ndim], [ilo[d] + N[d] - 1 for d in range(ndim)], 2, [0.05] * ndim,
                       [0.1, -0.15, 0.0][:ndim])
    rng = np.random.default_rng(M + ndim + ghost)
    lo, hi = np.array(geom.x_lower), np.array(geom.x_upper)
    X = rng.uniform(lo - 0.1 * (hi - lo), hi + 0.1 * (hi - lo), (M, ndim))
    if M:
        k = max(1, M // 20)
        X[:k] = lo + np.round((X[:k] - lo) / 0.05) * 0.05
    lag = (rng.permutation(M) * 2).astype(np.int32)
    if M > 100:
        lag[50:60] = lag[:10]
        X[50:60] = X[:10]  # the same node twice in one cell: numbered once
    order, nl, ng = le.node_distribution(ctx, geom, torch.from_numpy(X).cuda(), ghost,
                                         lag=torch.from_numpy(lag).cuda())
    eo, enl, eng = ora.node_distribution(X, geom.x_lower, geom.x_upper, geom.dx, geom.ilower, geom.iupper, ghost,
                                         lag=lag)
    assert (nl, ng) == (enl, eng)
    assert np.array_equal(order.cpu().numpy(), eo)


@pytest.mark.parametrize("ndim", [2, 3])
def test_order_is_independent_of_storage_order(le, ctx, ndim):
    """A reshuffled local storage (migrate(cell_order=False) appends arrivals) gives
    the same Lagrangian-index sequences: the lists and the numbering depend on the
    markers, not on where they are stored."""
    geom, X, lag = _case(le, ndim, 20000, 31, dup_lag=False)
    perm = np.random.default_rng(2).permutation(X.shape[0])
    seqs = []
    for P in (np.arange(X.shape[0]), perm):
        Xd = torch.from_numpy(X[P].copy()).cuda()
        lg = torch.from_numpy(lag[P].copy()).cuda()
        idx, xs = le.index_set_list(ctx, geom, Xd, 3, lag=lg)
        order, nl, ng = le.node_distribution(ctx, geom, Xd, 3, lag=lg)
        seqs.append((lag[P][idx.cpu().numpy()], xs.cpu().numpy(), lag[P][order.cpu().numpy()], nl, ng))
    a, b = seqs
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])
    assert np.array_equal(a[2], b[2]) and a[3:] == b[3:]


def test_index_list_after_slab_migration(le, ctx):
    """Markers re-owned by slab.migrate(cell_order=False) on one rank (P = 1: the
    wrap into the periodic box and the stayers-first layout) give the oracle's
    lists on the wrapped positions."""
    from ibamr_amd.slab import Slab, migrate
    slab = Slab([16, 16, 16], 1, 0, 3)
    geom = slab.geometry()
    rng = np.random.default_rng(8)
    M = 4000
    X = rng.uniform(-0.2, 1.2, (M, 3))
    lag = torch.from_numpy(rng.permutation(M).astype(np.int64))
    Xm, (lm,) = migrate(slab, torch.from_numpy(X).cuda(), [lag.cuda()], cell_order=False)
    lm32 = lm.to(torch.int32).contiguous()
    idx, xs = le.index_set_list(ctx, geom, Xm.contiguous(), 3, lag=lm32)
    Xn, ln = Xm.cpu().numpy(), lm32.cpu().numpy()
    ei, ex, _ = ora.periodic_index_list(Xn, geom.x_lower, geom.x_upper, geom.dx, geom.ilower, geom.iupper, 3, lag=ln)
    assert np.array_equal(idx.cpu().numpy(), ei) and np.array_equal(xs.cpu().numpy(), ex)
