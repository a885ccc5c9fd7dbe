"""GPU: the 3-D sweeps' work items do not change what is computed.

The segment length (ctx_tune "seg_items"), the load split of heavy (column,
segment) pairs ("split_target") and the heavy-first schedule ("heavy") only
regroup the same sweep.  Interp must be bitwise equal across settings and to
the oracle; spread must match the oracle within 1e-12 under every setting and be
bit-stable on a repeat.  (Spread sums may differ in the last bits between
settings: same-point adds inside one 64-candidate chunk follow its step and lane
order, and the chunk boundaries move with the items -- see le_sweep.hip.)
Segment lengths from 32 planes to the whole patch, uniform and clustered."""
import numpy as np
import pytest

from oracle import oracle as ora

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

SETTINGS = [
    {},                                                   # defaults
    {"seg_items": 64},                                    # one segment: the whole patch
    {"seg_items": 100000},                                # shortest segments (32 planes)
    {"seg_items": 2000, "split_target": 300},             # many load splits
    {"seg_items": 3000, "split_target": 500, "heavy": 1}, # every item heavy (scheduled first)
    {"heavy": -1},                                        # no heavy-first ordering
    {"xcd_block": 1},                                     # light items round-robin over the XCDs
    {"xcd_block": 3},                                     # ... in blocks of 3 table entries
]


@pytest.fixture(scope="module")
def le():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from ibamr_amd import le as _le
    return _le


def _markers(kind, M, rng):
    if kind == "uniform":
        return rng.uniform(0.0, 1.0, (M, 3))
    X = rng.uniform(0.0, 1.0, (M, 3))
    X[: M // 2, 2] = 0.37 + (X[: M // 2, 2] - 0.5) / 96.0  # a sheet one cell thick
    r = 0.03 * np.sqrt(X[M // 2:, 0])
    t = 2 * np.pi * X[M // 2:, 1]
    X[M // 2:, 0] = 0.6 + r * np.cos(t)                     # a bundle along z
    X[M // 2:, 1] = 0.45 + r * np.sin(t)
    return X


@pytest.mark.parametrize("kind", ["uniform", "clustered"])
def test_item_settings_do_not_change_results(le, kind):
    N = (96, 80, 112)
    geom = le.Geometry.periodic_unit(list(N), 3)
    rng = np.random.default_rng(21)
    M = 60000
    Xn = _markers(kind, M, rng)
    F = rng.standard_normal((M, 3))
    u = geom.alloc("side")
    for a in u:
        a.copy_(torch.from_numpy(rng.uniform(-1, 1, tuple(a.shape))))
    u0 = [a.cpu().numpy().copy() for a in u]
    X = torch.from_numpy(Xn).cuda()
    Fd = torch.from_numpy(F).cuda()
    idx = np.arange(M, dtype=np.int32)
    xs = np.zeros((M, 3))
    Uo = np.zeros((M, 3))
    ora.side_interp("IB_4", geom.dx, geom.x_lower, geom.ilower, geom.iupper, geom.gcw, u0, idx, xs, Xn, Uo)
    fo = None
    for st in SETTINGS:
        ctx = le.Context(0)
        for k, v in st.items():
            ctx.tune(k, v)
        m = le.Markers(ctx).bin(geom, "IB_4", X)
        U = torch.zeros((M, 3), dtype=torch.float64, device="cuda")
        le.interp(ctx, m, "IB_4", "side", geom, u, U, X)
        runs = []
        for rep in range(2):
            f = geom.alloc("side")
            le.spread(ctx, m, "IB_4", "side", geom, f, Fd, X)
            runs.append(f)
        ctx.synchronize()
        assert np.array_equal(U.cpu().numpy(), Uo), st  # interp: bitwise, every setting
        for a in range(3):
            assert torch.equal(runs[0][a], runs[1][a]), (st, a)  # spread: bit-stable
        if fo is None:  # the oracle in the binned order (the same under every setting)
            order = m.order().cpu().numpy()
            fo = [np.zeros_like(a) for a in u0]
            ora.side_spread("IB_4", geom.dx, geom.x_lower, geom.ilower, geom.iupper, geom.gcw, fo, idx[order], xs, Xn,
                            F)
        for a in range(3):
            d = np.abs(runs[0][a].cpu().numpy() - fo[a]).max() / np.abs(fo[a]).max()
            assert d <= 1e-12, (st, a, d)
