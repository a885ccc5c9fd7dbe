"""Checks of slab.redistribute's multi-rank numbering against the oracle (shared by the
gloo CPU test and the GPU migration test).  The oracle is the checker only."""
import numpy as np

from oracle import oracle as ora


def slab_boxes(N, P):
    nz = N[2] // P
    return [([0, 0, r * nz], [N[0] - 1, N[1] - 1, (r + 1) * nz - 1]) for r in range(P)]


def check_node_distribution(res, X_all, lag_all, N, P, ghost):
    """res: per rank, sorted by rank: dicts with lag, offset, num_nodes, ghost_lag,
    ghost_petsc (numpy).  X_all / lag_all: every marker after migration (each on its
    owner).  The level is the P z-slabs of an N grid on the periodic unit cube, patch
    r on rank r.

    * global numbering == the oracle's LDataManager::computeNodeDistribution over the
      whole level with the slabs in rank order (one rank's loops, LDataManager.cpp:
      2874-2892), i.e. local order and computeNodeOffsets (:3029-3047) together;
    * each rank's nonlocal nodes == the oracle's nonlocal walk over that rank's slab
      with every marker of the level visible (:2914-2944), and each carries the global
      index of its owner's node (AOApplicationToPetsc, :2995-3000)."""
    dx = [1.0 / n for n in N]
    boxes = slab_boxes(N, P)
    dom_hi = [n - 1 for n in N]
    eo, enl, enn = ora.level_node_distribution(X_all, lag_all, boxes, [0, 0, 0], dom_hi, [0.0] * 3, dx, 0)
    assert enn == 0 and enl == len(lag_all)
    glob = np.concatenate([r["lag"] for r in res])
    assert np.array_equal(glob, np.asarray(lag_all)[eo]), "global numbering differs from the oracle"
    off = 0
    for r in res:
        assert r["offset"] == off and r["num_nodes"] == enl, (r["offset"], off, r["num_nodes"], enl)
        off += len(r["lag"])
    petsc_of = {int(l): i for i, l in enumerate(glob)}
    n_ghost = 0
    for q, r in enumerate(res):
        o, nl, nn = ora.level_node_distribution(X_all, lag_all, [boxes[q]], [0, 0, 0], dom_hi, [0.0] * 3, dx, ghost)
        assert np.array_equal(np.asarray(lag_all)[o[:nl]], r["lag"]), f"rank {q}: local nodes"
        assert np.array_equal(np.asarray(lag_all)[o[nl:]], r["ghost_lag"]), f"rank {q}: nonlocal nodes"
        assert np.array_equal(r["ghost_petsc"], np.array([petsc_of[int(l)] for l in r["ghost_lag"]], dtype=np.int64))
        n_ghost += nn
    return n_ghost
