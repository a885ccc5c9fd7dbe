"""GPU: the fused ghost operations equal the unfused sequences bit for bit.

ibtk_le_zero_ghosts_spread = ibtk_le_zero_ghosts, then ibtk_le_spread: the 3-D
sweep's items start their owned ghost points from 0 and items no marker reaches
store the zeros.  Arrays start with NaN in their ghost layers (every ghost point must
be written, none read) and random interior values (kept and added to); markers cover
part of the patch only, so that ghost-owning items without candidates occur; every
kernel family and centering, packed and pitched layouts, an index list with periodic
images."""
import zlib

import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

from test_gpu_parity import make_case  # noqa: E402


@pytest.fixture(scope="module")
def le():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from ibamr_amd import le as _le
    return _le


@pytest.fixture(scope="module")
def ctx(le):
    return le.Context(0)


def _fill(q, geom, centering, rng):
    """random values, NaN in the ghost layers"""
    g = geom.gcw
    for c, a in enumerate(q):
        v = rng.uniform(-1, 1, tuple(a.shape))
        ext = geom.ext_mask(centering, c)
        mask = np.ones(a.shape[-3:] if geom.ndim == 3 else a.shape[-2:], bool)
        n = [geom.iupper[d] - geom.ilower[d] + 1 + ((ext >> d) & 1) for d in range(geom.ndim)]
        inner = tuple(slice(g[d], g[d] + n[d]) for d in reversed(range(geom.ndim)))
        mask[inner] = False
        v[..., mask] = np.nan
        a.copy_(torch.from_numpy(v))


@pytest.mark.parametrize("kernel,centering", [("IB_4", "side"), ("IB_6", "side"), ("PIECEWISE_LINEAR", "side"),
                                              ("IB_4", "cell"), ("IB_3", "node"), ("PIECEWISE_CUBIC", "edge"),
                                              ("BSPLINE_4", "side"), ("IB_4_W8", "cell")])
@pytest.mark.parametrize("pitched", [False, True])
def test_zero_ghosts_spread_equals_two_calls(le, ctx, kernel, centering, pitched):
    geom, X, idx, xs, depth = make_case(kernel, 3, centering, seed=zlib.crc32(f"zg{kernel}{centering}".encode()), M=400)
    if pitched:
        geom = geom.aligned()
    rng = np.random.default_rng(31)
    # markers in the lower half of the patch only: the upper items own ghosts and no candidates
    L2 = (geom.iupper[2] - geom.ilower[2] + 1) * geom.dx[2]
    X[:, 2] = np.minimum(X[:, 2], geom.x_lower[2] + 0.45 * L2)
    dev = "cuda:0"
    Xd, idd, xsd = torch.from_numpy(X).to(dev), torch.from_numpy(idx).to(dev), torch.from_numpy(xs).to(dev)
    Qd = 3 if centering in ("side", "edge") else depth
    F = torch.from_numpy(rng.uniform(-1, 1, (X.shape[0], Qd))).to(dev)
    m = le.Markers(ctx).bin(geom, kernel, Xd, idd, xsd)
    qa = geom.alloc(centering, depth)
    _fill(qa, geom, centering, rng)
    qb = geom.alloc(centering, depth)  # the same layout (pitched arrays are strided views)
    for a, b in zip(qa, qb):
        b.copy_(a)
    le.zero_ghosts(ctx, geom, centering, qa, q_depth=depth)
    le.spread(ctx, m, kernel, centering, geom, qa, F, Xd, q_depth=depth)
    le.zero_ghosts_spread(ctx, m, kernel, centering, geom, qb, F, Xd, q_depth=depth)
    ctx.synchronize()
    for a, b in zip(qa, qb):
        assert not torch.isnan(b).any(), "a ghost point was left unwritten"
        assert torch.equal(a, b)


@pytest.mark.parametrize("kernel,centering", [("IB_4", "side"), ("IB_6", "side"), ("PIECEWISE_CUBIC", "side"),
                                              ("IB_4", "cell"), ("IB_3", "node"), ("IB_4", "edge"),
                                              ("BSPLINE_4", "side"), ("IB_4_W8", "cell")])
@pytest.mark.parametrize("periodic", [(1, 1, 1), (1, 1, 0)])
def test_fill_interp_equals_two_calls(le, ctx, kernel, centering, periodic):
    """ibtk_le_fill_interp = ibtk_le_fill_periodic_ghosts then ibtk_le_interp, Q bit for
    bit; the fused call reads no ghost value (they are NaN in its arrays, except in the
    non-periodic dims, where the fill copies nothing either) and writes none."""
    geom, X, idx, xs, depth = make_case(kernel, 3, centering, seed=zlib.crc32(f"fi{kernel}{centering}".encode()), M=500)
    rng = np.random.default_rng(41)
    dev = "cuda:0"
    Xd, idd, xsd = torch.from_numpy(X).to(dev), torch.from_numpy(idx).to(dev), torch.from_numpy(xs).to(dev)
    Qd = 3 if centering in ("side", "edge") else depth
    m = le.Markers(ctx).bin(geom, kernel, Xd, idd, xsd)
    qa = geom.alloc(centering, depth)
    for a in qa:
        a.copy_(torch.from_numpy(rng.uniform(-1, 1, tuple(a.shape))))
    qb = [a.clone() for a in qa]
    if periodic == (1, 1, 1):
        _fill(qb, geom, centering, rng)  # NaN ghosts, new interior values ...
        for a, b in zip(qa, qb):          # ... the same interior as qa
            mask = ~torch.isnan(b)
            a[mask] = b[mask]
    q_before = [b.clone() for b in qb]
    Qa = torch.full((X.shape[0], Qd), np.nan, dtype=torch.float64, device=dev)
    Qb = torch.full_like(Qa, np.nan)
    le.fill_periodic_ghosts(ctx, geom, centering, qa, q_depth=depth, periodic=list(periodic))
    le.interp(ctx, m, kernel, centering, geom, qa, Qa, Xd, q_depth=depth)
    le.fill_interp(ctx, m, kernel, centering, geom, qb, Qb, Xd, q_depth=depth, periodic=list(periodic))
    ctx.synchronize()
    listed = np.zeros(X.shape[0], bool)
    listed[idx] = True
    a, b = Qa.cpu().numpy()[listed], Qb.cpu().numpy()[listed]
    assert np.array_equal(a, b), f"max diff {np.nanmax(np.abs(a - b))}"
    for b0, b1 in zip(q_before, qb):  # nothing written
        assert torch.equal(torch.nan_to_num(b0, nan=7.0), torch.nan_to_num(b1, nan=7.0))


@pytest.mark.parametrize("kernel,centering,ndim", [("IB_4", "side", 3), ("IB_6", "side", 3), ("PIECEWISE_LINEAR", "side", 3),
                                                   ("IB_4", "cell", 3), ("IB_3", "node", 3), ("PIECEWISE_CUBIC", "edge", 3),
                                                   ("BSPLINE_4", "side", 3), ("IB_4_W8", "cell", 3),
                                                   ("IB_4", "side", 2), ("IB_6", "cell", 2)])
@pytest.mark.parametrize("pitched", [False, True])
@pytest.mark.parametrize("empty", [False, True])
def test_zero_spread_equals_two_calls(le, ctx, kernel, centering, ndim, pitched, empty):
    """ibtk_le_zero_spread = every point of q to 0, then ibtk_le_spread (LDataManager::spread's
    target, LDataManager.cpp:596): q starts NaN everywhere in the fused call (no point may be
    read, every point must be written); markers cover part of the patch only, so that items
    without candidates occur; an empty list (the zeroing alone) and 2-D (the two steps)."""
    if pitched and ndim != 3:
        pytest.skip("pitched layouts are 3-D")
    geom, X, idx, xs, depth = make_case(kernel, ndim, centering, seed=zlib.crc32(f"zs{kernel}{centering}{ndim}".encode()),
                                        M=400)
    if pitched:
        geom = geom.aligned()
    if empty:
        idx = idx[:0]
        xs = xs[:0]
    rng = np.random.default_rng(53)
    a_ = ndim - 1  # markers in the lower half of the slowest dim
    L = (geom.iupper[a_] - geom.ilower[a_] + 1) * geom.dx[a_]
    X[:, a_] = np.minimum(X[:, a_], geom.x_lower[a_] + 0.45 * L)
    dev = "cuda:0"
    Xd, idd, xsd = torch.from_numpy(X).to(dev), torch.from_numpy(idx).to(dev), torch.from_numpy(xs).to(dev)
    Qd = ndim if centering in ("side", "edge") else depth
    F = torch.from_numpy(rng.uniform(-1, 1, (X.shape[0], Qd))).to(dev)
    m = le.Markers(ctx).bin(geom, kernel, Xd, idd, xsd)
    qa = geom.alloc(centering, depth)
    for a in qa:
        a.copy_(torch.from_numpy(rng.uniform(-1, 1, tuple(a.shape))))
    qb = geom.alloc(centering, depth)
    for a in qb:
        a.fill_(np.nan)
    for a in qa:
        a.zero_()
    le.spread(ctx, m, kernel, centering, geom, qa, F, Xd, q_depth=depth)
    le.zero_spread(ctx, m, kernel, centering, geom, qb, F, Xd, q_depth=depth)
    ctx.synchronize()
    for a, b in zip(qa, qb):
        assert not torch.isnan(b).any(), "a point was left unwritten"
        assert torch.equal(a, b)
    if empty:
        assert all(not b.any() for b in qb)
