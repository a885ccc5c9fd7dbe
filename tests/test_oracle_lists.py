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
