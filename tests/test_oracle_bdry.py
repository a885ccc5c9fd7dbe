"""Oracle: physical-boundary operators for side data.

oracle/le_bdry_oracle.c restates CartSideRobinPhysBdryOp's forward ghost fill
(setPhysicalBoundaryConditions, CartSideRobinPhysBdryOp.cpp:358-422) and its
adjoint fold (accumulateFromPhysicalBoundaryData, :429-493) with the arithmetic
of cartphysbdryop{2,3}d.f.m4.  The Fortran cannot be built here and the
reference holds no fixtures for it, so the restatement is pinned by:

* transposition: with homogeneous Robin data (b != 0, g = 0) the adjoint is the
  exact transpose of the fill, <f, L u> = <L^T f, u> over the interior, for every
  mix of physical faces (faces, edges, corners);
* hand-worked values of each formula (Dirichlet reflection, Robin weights,
  linear extrapolation of edges and corners, the 3-D dx(location_index/NDIM) quirk);
* the Dirichlet adjoint's overwrite of the boundary value (f.m4:890-899).
"""
import numpy as np
import pytest

from oracle import oracle as ora


def _arrays(lo, hi, g, rng=None, fill=0.0):
    nd = len(lo)
    out = []
    for a in range(nd):
        shp = ora.side_ghost_shape(lo, hi, g, a)
        out.append(rng.standard_normal(shp) if rng is not None else np.full(shp, fill))
    return out


def _interior_mask(lo, hi, g, a, phys):
    """Points the fill never writes: side indices inside the patch (the upper
    face included), and the normal component's boundary faces when they are
    Robin (read, not written)."""
    nd = len(lo)
    shp = ora.side_ghost_shape(lo, hi, g, a)
    m = np.ones(shp, dtype=bool)
    for d in range(nd):
        ax = nd - 1 - d  # numpy axis of dim d
        n = hi[d] - lo[d] + 1 + (1 if d == a else 0)
        idx = np.arange(shp[ax])
        inside = (idx >= g) & (idx < g + n)
        sl = [None] * nd
        sl[ax] = slice(None)
        m &= inside[tuple(sl)]
    return m


CASES = [
    ([0, 0], [6, 5], 2),
    ([0, 0], [7, 7], 3),
    ([2, -1], [9, 6], 1),
    ([0, 0, 0], [5, 4, 6], 2),
    ([1, 0, -2], [6, 6, 3], 3),
]


@pytest.mark.parametrize("lo,hi,g", CASES)
@pytest.mark.parametrize("pattern", ["all", "mixed", "one"])
def test_adjoint_is_transpose_robin(lo, hi, g, pattern):
    nd = len(lo)
    rng = np.random.default_rng(7 + len(lo) + g)
    phys = {"all": [1] * (2 * nd), "mixed": [1, 0, 0, 1, 1, 1][:2 * nd], "one": [0, 0, 1, 0, 0, 0][:2 * nd]}[pattern]
    dx = [0.1, 0.13, 0.07][:nd]
    A = rng.uniform(0.5, 2.0, (nd, 2 * nd))
    B = rng.uniform(0.5, 2.0, (nd, 2 * nd))
    G = np.zeros((nd, 2 * nd))
    masks = [_interior_mask(lo, hi, g, a, phys) for a in range(nd)]
    # L u: interior random, ghosts zero, then the fill
    u = _arrays(lo, hi, g, rng)
    for a in range(nd):
        u[a][~masks[a]] = 0.0
    Lu = [x.copy() for x in u]
    ora.phys_bdry_side(lo, hi, g, dx, Lu, phys, A, B, G, adjoint=False)
    f = _arrays(lo, hi, g, rng)
    Ltf = [x.copy() for x in f]
    ora.phys_bdry_side(lo, hi, g, dx, Ltf, phys, A, B, G, adjoint=True)
    lhs = sum(float(np.sum(f[a] * Lu[a])) for a in range(nd))
    rhs = sum(float(np.sum(Ltf[a][masks[a]] * u[a][masks[a]])) for a in range(nd))
    assert abs(lhs - rhs) <= 1e-11 * max(1.0, abs(lhs)), (lhs, rhs)
    # and the fill did write ghosts of every physical face (the identity is not vacuous)
    assert any(np.any(Lu[a][~masks[a]] != 0) for a in range(nd))


def test_fill_formulas_2d_by_hand():
    lo, hi, g = [0, 0], [4, 3], 2
    dx = [0.25, 0.5]
    rng = np.random.default_rng(3)
    u = _arrays(lo, hi, g, rng)
    u0 = [x.copy() for x in u]
    phys = [1, 0, 0, 1]  # x-lower, y-upper
    A = np.array([[2.0, 1, 1, 3.0], [1.5, 1, 1, 0.5]])
    B = np.array([[0.0, 1, 1, 0.25], [0.75, 1, 1, 0.0]])
    G = np.array([[0.6, 0, 0, 0.2], [0.3, 0, 0, 0.9]])
    ora.phys_bdry_side(lo, hi, g, dx, u, phys, A, B, G, adjoint=False)
    # u0 (numpy index [j + g, i + g]); x-lower face, normal comp 0, Dirichlet (b = 0)
    ub = G[0, 0] / A[0, 0]
    for j in range(lo[1], hi[1] + 1):
        J = j + g
        assert u[0][J, 0 + g] == ub
        for i in range(1, g + 1):
            assert u[0][J, g - i] == -1.0 * u0[0][J, g + i] + 2.0 * ub
    # u1 on the x-lower face: transverse, cell-centred Robin (a, b, g) = (1.5, 0.75, 0.3), h = dx(0/2)
    a, b, gg, h = 1.5, 0.75, 0.3, dx[0]
    for j in range(lo[1], hi[1] + 2):  # side range of comp 1 (upper face included)
        J = j + g
        for i in range(g):
            n = 1.0 + 2.0 * i
            f_i = -(a * n * h - 2.0 * b) / (a * n * h + 2.0 * b)
            f_g = 2.0 * n * h / (a * n * h + 2.0 * b)
            # the source is read after the normal fills (which run first and set the
            # y-upper Dirichlet face of u1, j = hi + 1)
            assert u[1][J, g - 1 - i] == f_i * u[1][J, g + i] + f_g * gg
    # u1 on the y-upper face: normal comp 1, Dirichlet (b = 0): boundary index hi+1
    ub = G[1, 3] / A[1, 3]
    Jb = hi[1] + 1 + g
    for i0 in range(lo[0], hi[0] + 1):
        I = i0 + g
        assert u[1][Jb, I] == ub
        for k in range(1, g + 1):
            assert u[1][Jb + k, I] == -1.0 * u0[1][Jb - k, I] + 2.0 * ub
    # corner (x-lower, y-upper): u0 extrapolated linearly along y from the face ghosts
    jb = hi[1]
    for j in range(hi[1] + 1, hi[1] + g + 1):
        for i in range(lo[0] - g, lo[0]):
            d = float(abs(j - jb))
            exp = (1.0 + d) * u[0][jb + g, i + g] - d * u[0][jb - 1 + g, i + g]
            assert u[0][j + g, i + g] == exp


def test_edge_extrapolation_3d():
    """An x-edge ghost of u1 is the linear extrapolation along z of the face ghosts
    (scrobinphysbdryop23d), and the fill leaves the interior alone."""
    lo, hi, g = [0, 0, 0], [4, 5, 3], 2
    nd = 3
    us = []
    for a in range(nd):
        shp = ora.side_ghost_shape(lo, hi, g, a)
        k, j, i = np.meshgrid(*[np.arange(s) for s in shp], indexing="ij")
        us.append((0.5 + 1.0 * i + 2.0 * j + 4.0 * k).astype(np.float64))
    ref = [x.copy() for x in us]
    # homogeneous Neumann (a = 0, b = 1, g = 0) on every face
    A = np.zeros((nd, 2 * nd))
    B = np.ones((nd, 2 * nd))
    G = np.zeros((nd, 2 * nd))
    ora.phys_bdry_side(lo, hi, g, [1.0, 1.0, 1.0], us, [1] * 6, A, B, G, adjoint=False)
    # an edge point of u1 (x-edge, lower y, lower z): extrapolated along z from the
    # (j ghost, k interior) face ghosts the codim-1 fill wrote before it
    i, j, k = 2, -1, -2
    kb = lo[2]
    I, J, K = i + g, j + g, k + g
    d = float(abs(k - kb))
    assert us[1][K, J, I] == (1.0 + d) * us[1][kb + g, J, I] - d * us[1][kb + 1 + g, J, I]
    # interior untouched
    m = _interior_mask(lo, hi, g, 1, [1] * 6)
    assert np.array_equal(us[1][m], ref[1][m])


def test_dx_location_quirk_3d():
    """h = dx(location_index/NDIM): in 3-D the y-lower face (loc 2) uses dx(0)."""
    lo, hi, g = [0, 0, 0], [3, 3, 3], 1
    A = np.ones((3, 6))
    B = np.ones((3, 6))
    G = np.zeros((3, 6))
    phys = [0, 0, 1, 0, 0, 0]
    dxa, dxb = [0.1, 0.2, 0.3], [0.1, 0.9, 0.9]
    out = []
    for dx in (dxa, dxb):
        u = _arrays(lo, hi, g, np.random.default_rng(5))
        ora.phys_bdry_side(lo, hi, g, dx, u, phys, A, B, G, adjoint=False)
        out.append(u)
    # only dx[0] matters for loc 2: changing dx[1], dx[2] changes nothing
    for a in range(3):
        assert np.array_equal(out[0][a], out[1][a])


def test_dirichlet_adjoint_overwrites_boundary_value():
    lo, hi, g = [0, 0], [3, 3], 2
    u = _arrays(lo, hi, g, np.random.default_rng(11))
    u_before = [x.copy() for x in u]
    A = np.full((2, 4), 2.0)
    B = np.zeros((2, 4))
    G = np.full((2, 4), 0.5)
    ora.phys_bdry_side(lo, hi, g, [1.0, 1.0], u, [1, 0, 0, 0], A, B, G, adjoint=True)
    for j in range(lo[1], hi[1] + 1):
        J = j + g
        exp = 0.5 / 2.0
        for i in range(1, g + 1):
            exp = exp + 2.0 * u_before[0][J, g - i]
        assert u[0][J, g] == exp


def test_no_physical_faces_is_identity():
    for lo, hi, g in CASES:
        nd = len(lo)
        u = _arrays(lo, hi, g, np.random.default_rng(1))
        ref = [x.copy() for x in u]
        for adj in (False, True):
            ora.phys_bdry_side(lo, hi, g, [1.0] * nd, u, [0] * (2 * nd), 1.0, 1.0, 0.0, adjoint=adj)
        for a in range(nd):
            assert np.array_equal(u[a], ref[a])
