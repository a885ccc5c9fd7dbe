"""The oracle's USER_DEFINED restatement (LEInteractor::userDefinedInterpolate /
userDefinedSpread, LEInteractor.cpp:3141-3393) pinned against its independent
twin: with the reference's default kernel function (ib4_kernel_fcn, stencil 4,
LEInteractor.cpp:629-652) it must reproduce the IB_4 Fortran restatement
(lagrangian_interaction{2,3}d.f.m4) -- the same kernel reached through a floor-based
stencil rule and |r| weights instead of NINT and the closed form -- within rounding,
on side-centred data with clipped stencils.  Entries with a periodic shift are left
out of that comparison: the reference picks an even stencil by comparing the
UNSHIFTED X with the shifted cell centre (LEInteractor.cpp:3188), which the
restatement keeps, so an image's stencil may sit one cell off IB_4's.  A linear hat
kernel (stencil 2) interpolates linear fields exactly."""
import numpy as np
import pytest

from oracle import oracle as ora


def _side_case(nd, seed, M=200, shifts=True):
    rng = np.random.default_rng(seed)
    lo = [2, -1, 4][:nd]
    hi = [lo[d] + 9 + d for d in range(nd)]
    g = [3] * nd
    dx = [0.1, 0.08, 0.06][:nd]
    xl = [-0.2, 0.3, 1.1][:nd]
    L = np.array([(hi[d] - lo[d] + 1) * dx[d] for d in range(nd)])
    X = xl + rng.uniform(-0.15, 1.15, (M, nd)) * L
    idx = np.arange(M, dtype=np.int32)
    xs = np.zeros((M, nd))
    pick = (rng.random(M) < 0.25) & shifts
    xs[pick] = rng.integers(-1, 2, (pick.sum(), nd)) * L
    u = [rng.uniform(-1, 1, ora.ghost_shape(*ora.side_box(lo, hi, a), g)) for a in range(nd)]
    return lo, hi, g, dx, xl, X, idx, xs, u


@pytest.mark.parametrize("nd", [2, 3])
def test_user_default_reproduces_ib4(nd):
    ora.set_user_kernel(None, 4)
    lo, hi, g, dx, xl, X, idx, xs, u = _side_case(nd, 7 + nd, shifts=False)
    Qu, Qi = np.zeros((X.shape[0], nd)), np.zeros((X.shape[0], nd))
    ora.side_interp("USER_DEFINED", dx, xl, lo, hi, g, u, idx, xs, X, Qu)
    ora.side_interp("IB_4", dx, xl, lo, hi, g, u, idx, xs, X, Qi)
    assert np.abs(Qu - Qi).max() <= 1e-13 * np.abs(Qi).max()
    F = np.random.default_rng(1).uniform(-1, 1, (X.shape[0], nd))
    fu = [np.zeros_like(a) for a in u]
    fi = [np.zeros_like(a) for a in u]
    ora.side_spread("USER_DEFINED", dx, xl, lo, hi, g, fu, idx, xs, X, F)
    ora.side_spread("IB_4", dx, xl, lo, hi, g, fi, idx, xs, X, F)
    for a, b in zip(fu, fi):
        assert np.abs(a - b).max() <= 1e-12 * np.abs(b).max()


def test_user_hat_interpolates_linear_fields():
    def hat(r):
        r = abs(r)
        return 1.0 - r if r < 1.0 else 0.0
    ora.set_user_kernel(hat, 2)
    try:
        nd, lo, hi, g = 3, [0, 0, 0], [7, 7, 7], [2, 2, 2]
        dx, xl = [0.125] * 3, [0.0] * 3
        shape = ora.ghost_shape(lo, hi, g)
        # cell centres x_i = (i + 1/2) dx; u = 1 + 2x - 3y + 0.5z
        ii = [np.arange(lo[d] - g[d], hi[d] + g[d] + 1) for d in range(nd)]
        zc, yc, xc = np.meshgrid(*[(v + 0.5) * dx[d] for d, v in reversed(list(enumerate(ii)))], indexing="ij")
        u = (1.0 + 2.0 * xc - 3.0 * yc + 0.5 * zc).reshape(shape)
        rng = np.random.default_rng(2)
        X = rng.uniform(0.1, 0.9, (100, 3))
        idx = np.arange(100, dtype=np.int32)
        V = np.zeros(100)
        ora.interp("USER_DEFINED", dx, xl, lo, hi, g, u, idx, np.zeros((100, 3)), X, V)
        expect = 1.0 + 2.0 * X[:, 0] - 3.0 * X[:, 1] + 0.5 * X[:, 2]
        assert np.abs(V - expect).max() <= 1e-13
    finally:
        ora.set_user_kernel(None, 4)


def test_user_shift_quirk_kept():
    """An image (X + shift) whose unshifted X lies on the other side of its cell centre
    takes the other even stencil (LEInteractor.cpp:3188): the restatement keeps it, so
    its interp differs from IB_4's for such entries and only for them."""
    ora.set_user_kernel(None, 4)
    lo, hi, g, dx, xl, X, idx, xs, u = _side_case(3, 10)
    Qu, Qi = np.zeros((X.shape[0], 3)), np.zeros((X.shape[0], 3))
    ora.side_interp("USER_DEFINED", dx, xl, lo, hi, g, u, idx, xs, X, Qu)
    ora.side_interp("IB_4", dx, xl, lo, hi, g, u, idx, xs, X, Qi)
    differ = np.abs(Qu - Qi).max(axis=1) > 1e-12 * np.abs(Qi).max()
    assert differ.any() and not differ[np.all(xs == 0, axis=1)].any()
