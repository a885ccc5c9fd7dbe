"""CPU: the oracle's restatement of the index bookkeeping (LIndexSetData::
cacheLocalIndices, LIndexSetData.cpp:83-169; LDataManager::computeNodeDistribution,
LDataManager.cpp:2874-2947; the per-cell sort + unique, :1487-1493), on hand-made
cases whose answer can be read off."""
import numpy as np

from oracle import oracle as ora


def _geom(N=4):
    return [0.0, 0.0], [1.0, 1.0], [1.0 / N, 1.0 / N], [0, 0], [N - 1, N - 1]


def test_list_order_is_cell_then_lagrangian_index():
    xlo, xup, dx, lo, hi = _geom()
    # cells (x, y): m0 (1, 1), m1 (0, 2), m2 (1, 1), m3 (3, 0)
    X = np.array([[0.30, 0.30], [0.10, 0.60], [0.26, 0.40], [0.90, 0.10]])
    lag = np.array([9, 4, 2, 7])
    idx, xs, cells = ora.periodic_index_list(X, xlo, xup, dx, lo, hi, 0, lag=lag, which="interior")
    # box order, x fastest: (3,0) key 3, (1,1) key 5, (0,2) key 8; in (1,1): lag 2 (m2) before 9 (m0)
    assert idx.tolist() == [3, 2, 0, 1]
    assert not xs.any()
    idx2, _, _ = ora.periodic_index_list(X, xlo, xup, dx, lo, hi, 0, which="interior")
    assert idx2.tolist() == [3, 0, 2, 1]  # lag = marker index


def test_images_and_shifts():
    xlo, xup, dx, lo, hi = _geom()
    X = np.array([[0.10, 0.40]])  # cell (0, 1): one image at x cell 4 (ghost 1), shift +1 in x
    idx, xs, cells = ora.periodic_index_list(X, xlo, xup, dx, lo, hi, 1, which="all")
    assert idx.tolist() == [0, 0]
    assert cells.tolist() == [[0, 1], [4, 1]]
    assert xs.tolist() == [[0.0, 0.0], [1.0, 0.0]]
    gi, gx, _ = ora.periodic_index_list(X, xlo, xup, dx, lo, hi, 1, which="ghost")
    assert gi.tolist() == [0] and gx.tolist() == [[1.0, 0.0]]


def test_node_distribution_local_then_ghost_unique():
    xlo, xup, dx, lo, hi = [0.0, 0.0], [0.5, 1.0], [0.25, 0.25], [0, 0], [1, 3]
    X = np.array([[0.30, 0.30],   # local (1, 1)
                  [0.60, 0.10],   # ghost cell (2, 0)
                  [0.26, 0.35],   # local (1, 1)
                  [0.30, 0.30],   # local (1, 1) again, same Lagrangian index as m0
                  [1.50, 0.10]])  # beyond a 1-cell ghost box: not numbered
    lag = np.array([5, 1, 3, 5, 8])
    order, nl, ng = ora.node_distribution(X, xlo, xup, dx, lo, hi, 1, lag=lag)
    assert order.tolist() == [2, 0, 1] and (nl, ng) == (2, 1)


def test_index_set_list_uniques_lagrangian_duplicates():
    """Two markers of one cell with one Lagrangian index are one LNode: the set is
    sorted and uniqued (LDataManager.cpp:1487-1493), the lower marker index kept."""
    xlo, xup, dx, lo, hi = _geom()
    X = np.array([[0.30, 0.30], [0.26, 0.40], [0.31, 0.33], [0.90, 0.10]])  # m0, m1, m2 in cell (1, 1)
    lag = np.array([6, 2, 6, 1])
    idx, _, cells = ora.periodic_index_list(X, xlo, xup, dx, lo, hi, 0, lag=lag, which="all")
    assert idx.tolist() == [3, 1, 0]
    sets = ora.lnode_set_data(X, xlo, xup, dx, lo, hi, 0, lag=lag)
    assert sets[(1, 1)] == [1, 0] and sets[(3, 0)] == [3]


def test_build_local_indices_box_branch_by_hand():
    """LEInteractor.cpp:3070-3106 on a 4x4 periodic patch with 1 ghost cell: a box
    reaching one cell below the patch in x picks the image of the x = 3 column's
    marker at cell (-1, y) with offset -periodic_shift * dx, before the box's own cells."""
    xlo, xup, dx, lo, hi = _geom()
    X = np.array([[0.90, 0.40], [0.10, 0.40], [0.60, 0.90]])  # cells (3, 1), (0, 1), (2, 3)
    sets = ora.lnode_set_data(X, xlo, xup, dx, lo, hi, 1)
    idx, xs, cells = ora.build_local_indices(sets, dx, lo, hi, 1, ([-1, 0], [1, 2]))
    assert idx.tolist() == [0, 1]
    assert cells.tolist() == [[-1, 1], [0, 1]]
    assert xs.tolist() == [[-1.0, 0.0], [0.0, 0.0]]
    # a box above the patch in y: (2, 3) itself and nothing else; (2, 4) holds the image of (2, 0): none
    idx, xs, cells = ora.build_local_indices(sets, dx, lo, hi, 1, ([2, 3], [2, 4]))
    assert idx.tolist() == [2] and cells.tolist() == [[2, 3]] and not xs.any()


def test_build_local_indices_matches_cached_lists():
    """The cell-walk restatement of buildLocalIndices gives cacheLocalIndices' lists for
    box == patch box and box == ghost box, and their box-filtered entries for any other
    box (two independent derivations: offsets from the cell vs from the image shift)."""
    rng = np.random.default_rng(5)
    N, g = [6, 5, 7], 2
    lo, hi = [0, 0, 0], [N[0] - 1, N[1] - 1, N[2] - 1]
    dx = [1.0 / n for n in N]
    X = rng.uniform(0, 1, (70, 3))
    lag = rng.integers(0, 50, 70)  # repeated Lagrangian indices on purpose
    sets = ora.lnode_set_data(X, [0, 0, 0], [1, 1, 1], dx, lo, hi, g, lag=lag)
    ia, xa, ca = ora.periodic_index_list(X, [0, 0, 0], [1, 1, 1], dx, lo, hi, g, lag=lag, which="all")
    ii, xi, _ = ora.periodic_index_list(X, [0, 0, 0], [1, 1, 1], dx, lo, hi, g, lag=lag, which="interior")
    gb = ([lo[d] - g for d in range(3)], [hi[d] + g for d in range(3)])
    for box, (ei, ex) in (((lo, hi), (ii, xi)), (gb, (ia, xa))):
        bi, bx, _ = ora.build_local_indices(sets, dx, lo, hi, g, box)
        assert bi.tolist() == ei.tolist() and np.array_equal(bx, ex)
    for box in (([-2, 1, 0], [3, 6, 2]), ([4, -1, -2], [7, 3, 8]), ([1, 1, 1], [1, 1, 1])):
        bi, bx, bc = ora.build_local_indices(sets, dx, lo, hi, g, box)
        sel = np.all((ca >= np.array(box[0])) & (ca <= np.array(box[1])), axis=1)
        assert bi.tolist() == ia[sel].tolist() and np.array_equal(bx, xa[sel]) and np.array_equal(bc, ca[sel])


def test_level_node_distribution_by_hand():
    """Two 2x2 patches of a 4x2 periodic domain, patch order [right, left], one ghost
    cell: the right patch's nodes first (box order, Lagrangian order in a cell), then
    the left's; no nonlocal nodes (every marker is in a local patch)."""
    X = np.array([[0.10, 0.10],   # cell (0, 0): left patch
                  [0.60, 0.80],   # (2, 1): right
                  [0.90, 0.20],   # (3, 0): right
                  [0.65, 0.70]])  # (2, 1): right, Lagrangian index below marker 1's
    lag = np.array([0, 7, 5, 3])
    patches = [([2, 0], [3, 1]), ([0, 0], [1, 1])]
    order, nl, nn = ora.level_node_distribution(X, lag, patches, [0, 0], [3, 1], [0.0, 0.0], [0.25, 0.5], 1)
    assert order.tolist() == [2, 3, 1, 0] and (nl, nn) == (4, 0)
    # only the right patch is local: the left's marker is a nonlocal node of its ghost cells
    # (cell (1, .) left of it is ghost, and (0, 0)'s periodic image (4, 0) right of it)
    order, nl, nn = ora.level_node_distribution(X, lag, patches[:1], [0, 0], [3, 1], [0.0, 0.0], [0.25, 0.5], 1)
    assert order.tolist() == [2, 3, 1, 0] and (nl, nn) == (3, 1)
