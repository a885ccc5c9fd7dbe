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
