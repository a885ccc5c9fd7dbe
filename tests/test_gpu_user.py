"""GPU parity of the USER_DEFINED kernel function (LEInteractor::userDefinedInterpolate /
userDefinedSpread, LEInteractor.cpp:3141-3393) through ibtk_le_user_interp / _spread,
against the oracle's restatement (oracle/le_oracle.c ora_user_call) with the same host
kernel function: both the interp (the reference's loop order, the last entry naming a
marker writes it) and the spread (every grid point summed in list order) are expected
bit for bit.  Kernel functions: the reference's default (IB_4's ib4_kernel_fcn,
stencil 4), the re-scaled IB_4 kernel of the reference's example ex4 (width 6), and a
3-point and a 6-point polynomial one (+ and * only).  The host evaluates the kernel
function for both sides (the library through a ctypes callback into the same Python
function), so the weights are the same bits."""
import zlib

import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

from test_gpu_parity import make_case, oracle_call, rel_err  # noqa: E402


def phi3(r):  # a 3-point kernel: (9/4 - r^2)/4 inside |r| < 3/2
    r2 = r * r
    return (2.25 - r2) * 0.25 if r2 < 2.25 else 0.0


def phi6(r):  # a 6-point kernel: (9 - r^2)^2 / 81 / 4.2 inside |r| < 3
    r2 = r * r
    t = 9.0 - r2
    return t * t / 340.2 if r2 < 9.0 else 0.0


def scaled_ib4_W6(r):  # the reference's own user kernel (examples/IB/explicit/ex4/main.cpp:88-96), W = 6
    from oracle.oracle import ib4_kernel_fcn
    return ib4_kernel_fcn(r / (6.0 / 4.0)) / (6.0 / 4.0)


KERNELS = {"default": (None, 4), "phi3": (phi3, 3), "phi6": (phi6, 6), "ex4_W6": (scaled_ib4_W6, 6)}
CASES = [(k, nd, c) for k in KERNELS for nd in (2, 3) for c in ("side", "cell", "node", "edge")
         if not (c == "edge" and nd == 2)]


@pytest.fixture(scope="module")
def le():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from ibamr_amd import le as _le
    return _le


@pytest.fixture(scope="module")
def ctx(le):
    return le.Context(0)


@pytest.fixture(scope="module")
def oracle():
    from oracle import oracle as ora
    return ora


def _use(le, oracle, name):
    fn, S = KERNELS[name]
    le.set_user_kernel(fn, S)
    oracle.set_user_kernel(fn, S)


def _case(name, nd, cent, seed):
    geom, X, idx, xs, depth = make_case("USER_DEFINED", nd, cent, seed=seed)
    # entries naming a marker twice (the interp's last entry writes it; the spread adds both)
    idx = np.concatenate([idx, idx[:7]]).astype(np.int32)
    xs = np.concatenate([xs, xs[:7]])
    return geom, X, idx, xs, depth


@pytest.mark.parametrize("name,nd,cent", CASES, ids=lambda v: str(v))
def test_user_interp_matches_oracle(le, ctx, oracle, name, nd, cent):
    _use(le, oracle, name)
    try:
        geom, X, idx, xs, depth = _case(name, nd, cent, zlib.crc32(f"u{name}{nd}{cent}".encode()))
        rng = np.random.default_rng(3)
        dev = "cuda:0"
        q = geom.alloc(cent, depth)
        for a in q:
            a.copy_(torch.from_numpy(rng.uniform(-1, 1, tuple(a.shape))))
        Qdepth = nd if cent in ("side", "edge") else depth
        Q = torch.full((X.shape[0], Qdepth), np.nan, dtype=torch.float64, device=dev)
        le.user_interp(ctx, cent, geom, q, Q, torch.from_numpy(X).to(dev), torch.from_numpy(idx).to(dev),
                       torch.from_numpy(xs).to(dev), q_depth=depth)
        ctx.synchronize()
        Qg = Q.cpu().numpy()
        Qo = np.full_like(Qg, np.nan)
        oracle_call(oracle, "interp", "USER_DEFINED", cent, geom, [a.cpu().numpy().copy() for a in q], idx, xs, X,
                    Qo, depth)
        listed = np.zeros(X.shape[0], bool)
        listed[idx] = True
        assert np.isnan(Qg[~listed]).all(), "unlisted markers must be untouched"
        assert np.array_equal(Qg[listed], Qo[listed]), f"interp rel err {rel_err(Qg[listed], Qo[listed]):.3e}"
    finally:
        le.set_user_kernel(None, 4)
        oracle.set_user_kernel(None, 4)


@pytest.mark.parametrize("name,nd,cent", CASES, ids=lambda v: str(v))
def test_user_spread_matches_oracle(le, ctx, oracle, name, nd, cent):
    _use(le, oracle, name)
    try:
        geom, X, idx, xs, depth = _case(name, nd, cent, 1 + zlib.crc32(f"u{name}{nd}{cent}".encode()))
        rng = np.random.default_rng(4)
        dev = "cuda:0"
        q = geom.alloc(cent, depth)
        for a in q:
            a.copy_(torch.from_numpy(rng.uniform(-1, 1, tuple(a.shape))))
        u0 = [a.cpu().numpy().copy() for a in q]
        Qdepth = nd if cent in ("side", "edge") else depth
        F = rng.uniform(-1, 1, (X.shape[0], Qdepth))
        for _ in range(2):  # bit-stable: the second call adds the same again
            le.user_spread(ctx, cent, geom, q, torch.from_numpy(F).to(dev), torch.from_numpy(X).to(dev),
                           torch.from_numpy(idx).to(dev), torch.from_numpy(xs).to(dev), q_depth=depth)
            ctx.synchronize()
            oracle_call(oracle, "spread", "USER_DEFINED", cent, geom, u0, idx, xs, X, F.copy(), depth)
            for a, b in zip(q, u0):
                ag = a.cpu().numpy()
                assert np.array_equal(ag, b), f"spread rel err {rel_err(ag, b):.3e}"
    finally:
        le.set_user_kernel(None, 4)
        oracle.set_user_kernel(None, 4)


def test_user_default_is_ib4(le, ctx):
    """USER_DEFINED with the reference's default kernel function (ib4_kernel_fcn,
    stencil 4) against the IB_4 sweep path: the same kernel by a different stencil
    rule and weight formula, equal within rounding (interp 1e-13, spread 1e-12)."""
    le.set_user_kernel(None, 4)
    geom, X, idx, xs, depth = make_case("IB_4", 3, "side", seed=21, M=500, shifts=False)  # see test_oracle_user
    rng = np.random.default_rng(5)
    dev = "cuda:0"
    q = geom.alloc("side", 1)
    for a in q:
        a.copy_(torch.from_numpy(rng.uniform(-1, 1, tuple(a.shape))))
    Xd, idd, xsd = torch.from_numpy(X).to(dev), torch.from_numpy(idx).to(dev), torch.from_numpy(xs).to(dev)
    Qu = torch.zeros((X.shape[0], 3), dtype=torch.float64, device=dev)
    Qi = torch.zeros_like(Qu)
    le.user_interp(ctx, "side", geom, q, Qu, Xd, idd, xsd)
    m = le.Markers(ctx).bin(geom, "IB_4", Xd, idd, xsd)
    le.interp(ctx, m, "IB_4", "side", geom, q, Qi, Xd)
    ctx.synchronize()
    assert rel_err(Qu.cpu().numpy(), Qi.cpu().numpy()) <= 1e-13
    F = torch.from_numpy(rng.uniform(-1, 1, (X.shape[0], 3))).to(dev)
    fu, fi = geom.alloc("side", 1), geom.alloc("side", 1)
    le.user_spread(ctx, "side", geom, fu, F, Xd, idd, xsd)
    le.spread(ctx, m, "IB_4", "side", geom, fi, F, Xd)
    ctx.synchronize()
    for a, b in zip(fu, fi):
        assert rel_err(a.cpu().numpy(), b.cpu().numpy()) <= 1e-12


def phi20(r):  # a 20-point kernel: (100 - r^2)^2 / 53333.33.. inside |r| < 10 (past round 3's cap of 16)
    r2 = r * r
    t = 100.0 - r2
    return t * t / 53333.0 if r2 < 100.0 else 0.0


@pytest.mark.parametrize("op", ["interp", "spread"])
def test_user_wide_stencil(le, ctx, oracle, op):
    """Stencil size 20 (the reference takes any s_kernel_fcn_stencil_size,
    LEInteractor.cpp:652, 678): bitwise the oracle, 3-D side data."""
    le.set_user_kernel(phi20, 20)
    oracle.set_user_kernel(phi20, 20)
    try:
        geom, X, idx, xs, depth = make_case("IB_4", 3, "side", seed=77, M=60, extra_ghost=9)
        rng = np.random.default_rng(8)
        dev = "cuda:0"
        q = geom.alloc("side", 1)
        for a in q:
            a.copy_(torch.from_numpy(rng.uniform(-1, 1, tuple(a.shape))))
        u0 = [a.cpu().numpy().copy() for a in q]
        Xd, idd, xsd = torch.from_numpy(X).to(dev), torch.from_numpy(idx).to(dev), torch.from_numpy(xs).to(dev)
        if op == "interp":
            Q = torch.zeros((X.shape[0], 3), dtype=torch.float64, device=dev)
            le.user_interp(ctx, "side", geom, q, Q, Xd, idd, xsd)
            ctx.synchronize()
            Qo = np.zeros((X.shape[0], 3))
            oracle_call(oracle, "interp", "USER_DEFINED", "side", geom, u0, idx, xs, X, Qo, 1)
            assert np.array_equal(Q.cpu().numpy()[idx], Qo[idx])
        else:
            F = rng.uniform(-1, 1, (X.shape[0], 3))
            le.user_spread(ctx, "side", geom, q, torch.from_numpy(F).to(dev), Xd, idd, xsd)
            ctx.synchronize()
            oracle_call(oracle, "spread", "USER_DEFINED", "side", geom, u0, idx, xs, X, F.copy(), 1)
            for a, b in zip(q, u0):
                assert np.array_equal(a.cpu().numpy(), b)
    finally:
        le.set_user_kernel(None, 4)
        oracle.set_user_kernel(None, 4)


def test_user_errors(le, ctx):
    from ibamr_amd import _lib
    with pytest.raises(_lib.IBTKLEError):
        le.set_user_kernel(phi3, 0)  # stencil size < 1
    le.set_user_kernel(phi6, 6)  # needs 4 ghosts to interpolate (floor(6/2) + 1)
    try:
        from ibamr_amd.le import Geometry
        geom = Geometry([0, 0, 0], [7, 7, 7], 3, [0.1] * 3, [0.0] * 3)
        q = geom.alloc("side", 1)
        X = torch.rand((10, 3), dtype=torch.float64, device="cuda:0") * 0.8
        Q = torch.zeros_like(X)
        with pytest.raises(_lib.IBTKLEError) as e:
            le.user_interp(ctx, "side", geom, q, Q, X)
        assert e.value.code == 2  # IBTK_LE_ERR_GHOST_WIDTH (LEInteractor.cpp:2416-2426)
    finally:
        le.set_user_kernel(None, 4)
