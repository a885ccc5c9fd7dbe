"""GPU: density-weighted spread f += S (F ds) (ibtk_le_spread_ds).

LDataManager::spread with ds_data (LDataManager.cpp:398-470) forms F_ds = F * ds
per marker and spreads that.  The library forms the product in the gather that
stages F, so spread_ds(F, ds) must equal spread(F * ds) bit for bit, and match the
oracle's spread of the numpy product within the spread tolerance.
"""
import numpy as np
import pytest

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


@pytest.mark.parametrize("ndim", [2, 3])
@pytest.mark.parametrize("kernel", ["IB_4", "BSPLINE_4"])
def test_spread_ds(le, ctx, oracle, ndim, kernel):
    from ibamr_amd.le import Geometry
    N = [24] * ndim
    geom = Geometry.periodic_unit(N, oracle.min_ghost_width(kernel))
    rng = np.random.default_rng(ndim)
    M = 3000
    Xn = rng.random((M, ndim))
    Fn = rng.standard_normal((M, ndim))
    dsn = rng.random(M) * 1e-3 + 1e-4
    X, F, ds = (torch.from_numpy(a).cuda() for a in (Xn, Fn, dsn))
    m = le.Markers(ctx).bin(geom, kernel, X)
    q1 = geom.alloc("side")
    le.spread(ctx, m, kernel, "side", geom, q1, F, X, ds=ds)
    q2 = geom.alloc("side")
    le.spread(ctx, m, kernel, "side", geom, q2, F * ds[:, None], X)
    ctx.synchronize()
    for a, b in zip(q1, q2):
        assert torch.equal(a, b)
    order = m.order().cpu().numpy()
    uo = [np.zeros(tuple(a.shape)) for a in q1]
    idx = np.arange(M, dtype=np.int32)
    oracle.side_spread(kernel, geom.dx, geom.x_lower, geom.ilower, geom.iupper, geom.gcw, uo, idx[order],
                       np.zeros((M, ndim)), Xn, Fn * dsn[:, None])
    for a in range(ndim):
        ref = uo[a]
        err = np.abs(q1[a].cpu().numpy() - ref).max() / max(np.abs(ref).max(), 1e-300)
        assert err <= SPREAD_TOL, (a, err)


def test_spread_ds_errors(le, ctx):
    from ibamr_amd.le import Geometry
    geom = Geometry.periodic_unit([16, 16, 16], 3)
    X = torch.rand((10, 3), dtype=torch.float64, device="cuda:0")
    m = le.Markers(ctx).bin(geom, "IB_4", X)
    q = geom.alloc("side")
    with pytest.raises(ValueError):
        le.spread(ctx, m, "IB_4", "side", geom, q, X, X, ds=torch.ones(9, dtype=torch.float64, device="cuda:0"))
