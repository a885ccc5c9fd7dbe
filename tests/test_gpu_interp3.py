"""GPU: k_interp3 (ctx_tune interp3 = 1) -- the three components of a one-patch interp item in
one workgroup, each marker read once and each Q record written whole -- gives the per-component
kernel's result bit for bit, and so the oracle's (f.m4:1366-1382 order): plain and fused
periodic fill, identity lists and index lists with periodic images (a marker named twice: the
last entry writes Q), clustered markers (rounds of 256 markers per group), IB_4 and BSPLINE_4."""
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


def _interp(le, tune, kernel, geom, u, X, fill, indices=None, xshift=None):
    ctx = le.Context(0)
    if tune:
        ctx.tune("interp3", 1)
    m = le.Markers(ctx).bin(geom, kernel, X, indices, xshift)
    U = torch.full((X.shape[0], 3), 5.0, dtype=torch.float64, device="cuda")
    if fill:
        le.fill_interp(ctx, m, kernel, "side", geom, u, U, X, periodic=[1, 1, 1])
    else:
        le.interp(ctx, m, kernel, "side", geom, u, U, X)
    ctx.synchronize()
    return U


@pytest.mark.parametrize("kernel", ["IB_4", "BSPLINE_4"])
@pytest.mark.parametrize("fill", [False, True])
@pytest.mark.parametrize("markers", ["uniform", "clustered"])
def test_interp3_bitwise(le, kernel, fill, markers):
    g = le._lib.load().ibtk_le_min_ghost_width(le.kernel_id(kernel))
    geom = le.Geometry.periodic_unit([96, 64, 72], g)
    rng = np.random.default_rng(17)
    M = 60000
    X = rng.uniform(0.0, 1.0, (M, 3))
    if markers == "clustered":  # a sheet one cell thick: dense anchor planes, several rounds a group
        X[:, 2] = 0.4 + (X[:, 2] - 0.5) / 72
    Xd = torch.from_numpy(X).cuda()
    u = geom.alloc("side")
    for a in u:
        a.copy_(torch.from_numpy(rng.standard_normal(tuple(a.shape))))
    a = _interp(le, False, kernel, geom, u, Xd, fill)
    b = _interp(le, True, kernel, geom, u, Xd, fill)
    assert torch.equal(a, b)


def test_interp3_index_list_with_images(le):
    """A periodic ghost-box list (markers near the faces listed again, shifted): the Q row of
    a marker named twice comes from its last entry, in both kernels."""
    kernel = "IB_4"
    g = le._lib.load().ibtk_le_min_ghost_width(le.kernel_id(kernel))
    geom = le.Geometry.periodic_unit([64, 64, 64], g)
    rng = np.random.default_rng(3)
    M = 40000
    X = torch.from_numpy(rng.uniform(0.0, 1.0, (M, 3))).cuda()
    idx, xs = le.periodic_index_list(le.Context(0), geom, X, g)
    u = geom.alloc("side")
    for arr in u:
        arr.copy_(torch.from_numpy(rng.standard_normal(tuple(arr.shape))))
    a = _interp(le, False, kernel, geom, u, X, False, idx, xs)
    b = _interp(le, True, kernel, geom, u, X, False, idx, xs)
    assert torch.equal(a, b)
