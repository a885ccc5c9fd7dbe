"""GPU: the device kernels' 1-D weights against the known-answer vectors of
tests/golden/kernel_weights.json (60-digit Decimal evaluations of the
reference's formulas, made by tests/golden/make_golden.py independently of both
the oracle and le_stencil.h).

The device stencil code (ibamr_amd/csrc/le_stencil.h) and the oracle
(oracle/le_oracle.c) restate the same Fortran, so a transcription slip common to
both would pass every GPU-vs-oracle parity test; this test pins the device side
directly.  Method: cell-centred data (no frame shift), dx = 1, x_lower = 0,
ilower = 0, so X_o_dx = x exactly; the marker's y (and z) sit at a cell centre;
u = 1 on the whole grid plane x-index j, 0 elsewhere.  Then V = w(j) times the
partition-of-unity sums of the other dims (1 up to rounding; 1 + 6e-15 for
IB_3, whose truncated Fortran constants are kept).  Every point of every
stencil is checked, and the points just outside it must give exactly 0.
"""
import json
from decimal import Decimal
from pathlib import Path

import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

GOLDEN = json.loads((Path(__file__).parent / "golden" / "kernel_weights.json").read_text())
KERNELS = sorted({c["kernel"] for c in GOLDEN["cases"]})


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
@pytest.mark.parametrize("kernel", KERNELS + ["DISCONTINUOUS_LINEAR-offaxis"])
def test_device_weights_known_answer(le, ctx, kernel, ndim):
    off = kernel.endswith("-offaxis")
    kname = kernel.replace("-offaxis", "")
    cases = [c for c in GOLDEN["cases"] if c["kernel"] == kname and c.get("axis_dim", True) != off]
    assert cases
    axis = 1 if off else 0
    g = 8
    nx, ny = 21, 4
    ilo = [0] * ndim
    ihi = [nx - 1] + [ny - 1] * (ndim - 1)
    geom = le.Geometry(ilo, ihi, g, [1.0] * ndim, [0.0] * ndim)
    M = len(cases)
    X = np.full((M, ndim), 1.5)
    X[:, 0] = [float(c["X_o_dx"]) for c in cases]
    Xd = torch.from_numpy(X).cuda()
    m = le.Markers(ctx).bin(geom, kname, Xd)
    jmin = min(c["ic_lower"] for c in cases) - 1
    jmax = max(c["ic_lower"] + len(c["w"]) for c in cases)
    assert jmin >= -g and jmax <= nx - 1 + g
    got = np.zeros((M, jmax - jmin + 1))
    u = geom.alloc("cell")
    Q = torch.zeros((M, 1), dtype=torch.float64, device="cuda:0")
    for j in range(jmin, jmax + 1):
        u[0].zero_()
        u[0][..., j + g] = 1.0  # the whole plane x-index j (x is the fastest array dim)
        le.interp(ctx, m, kname, "cell", geom, u, Q, Xd, q_depth=1, axis=axis)
        ctx.synchronize()
        got[:, j - jmin] = Q[:, 0].cpu().numpy()
    tol = 2e-14
    for i, c in enumerate(cases):
        w = np.array([float(Decimal(v)) for v in c["w"]])
        k0 = c["ic_lower"] - jmin
        np.testing.assert_allclose(got[i, k0:k0 + w.size], w, rtol=0, atol=tol,
                                   err_msg=f"{kernel} {ndim}-D at X_o_dx = {c['X_o_dx']}")
        outside = np.delete(got[i], np.arange(k0, k0 + w.size))
        assert not outside.any(), f"{kernel} {ndim}-D at {c['X_o_dx']}: weight outside the stencil"


# ---------------------------------------------------------------------------- 3-D side KAT
KAT3 = json.loads((Path(__file__).parent / "golden" / "kat3d_side_ib4.json").read_text())


def test_device_side_ib4_known_answer_3d(le, ctx):
    """The headline path end to end on tests/golden/kat3d_side_ib4.json: 3-D side-centred
    IB_4 interp and spread at markers inside the patch, in its ghost region (stencils
    clipped by the ghost box) and as periodic images (Xshift), one marker listed twice,
    against 50-digit decimal evaluations of the Fortran text and LEInteractor's side
    frame shifts (tests/golden/make_kat3d.py), independent of the oracle.  Interp within
    1e-14 of the decimal value, spread within 1e-13 (relative to the largest magnitude)."""
    k = KAT3
    g = k["gcw"]
    geom = le.Geometry(k["ilower"], k["iupper"], g, k["dx"], k["x_lower"])
    q = geom.alloc("side")
    for a in range(3):
        q[a].copy_(torch.tensor(k["u"][a], dtype=torch.float64))
    X = torch.tensor(k["X"], dtype=torch.float64).cuda()
    F = torch.tensor(k["F"], dtype=torch.float64).cuda()
    idx = torch.tensor(k["indices"], dtype=torch.int32).cuda()
    xs = torch.tensor(k["Xshift"], dtype=torch.float64).cuda()
    m = le.Markers(ctx).bin(geom, "IB_4", X, idx, xs)
    Q = torch.zeros_like(X)
    le.interp(ctx, m, "IB_4", "side", geom, q, Q, X)
    le.spread(ctx, m, "IB_4", "side", geom, q, F, X)
    ctx.synchronize()
    Qe = np.array(k["Q"])
    assert np.abs(Q.cpu().numpy() - Qe).max() <= 1e-14 * np.abs(Qe).max()
    for a in range(3):
        fe = np.array(k["f"][a])
        assert np.abs(q[a].cpu().numpy() - fe).max() <= 1e-13 * np.abs(fe).max(), f"spread comp {a}"


# ---------------------------------------------------------------------------- every kernel
from test_oracle_kernels import KAT_CASES, kat_arrays, kat_expected_f, kat_id  # noqa: E402


@pytest.mark.parametrize("case", KAT_CASES, ids=kat_id)
def test_device_known_answers_every_kernel(le, ctx, case):
    """The device path on tests/golden/kat_kernels.json: every reference kernel function,
    2-D and 3-D, cell / node / side / edge data, against the 50-digit decimal evaluations of
    the Fortran text (tests/golden/make_kat.py), independent of the oracle and of
    le_stencil.h.  Interp within 1e-14, spread within 1e-13 (relative to the largest
    magnitude)."""
    k = case
    nd, dep, cent = k["ndim"], k["depth"], k["centering"]
    geom = le.Geometry(k["ilower"], k["iupper"], k["gcw"], k["dx"], k["x_lower"])
    arrays, _ = kat_arrays(k)
    q = geom.alloc(cent, dep)
    for a, src in zip(q, arrays):
        a.copy_(torch.from_numpy(src))
    X = torch.tensor(k["X"], dtype=torch.float64).cuda()
    Qd = nd if cent in ("side", "edge") else dep
    F = torch.tensor(k["F"], dtype=torch.float64)[:, :Qd].contiguous().cuda()
    idx = torch.tensor(k["indices"], dtype=torch.int32).cuda()
    xs = torch.tensor(k["Xshift"], dtype=torch.float64).cuda()
    m = le.Markers(ctx).bin(geom, k["kernel"], X, idx, xs)
    Q = torch.zeros((X.shape[0], Qd), dtype=torch.float64, device="cuda")
    le.interp(ctx, m, k["kernel"], cent, geom, q, Q, X, q_depth=dep, axis=k["axis"])
    le.spread(ctx, m, k["kernel"], cent, geom, q, F, X, q_depth=dep, axis=k["axis"])
    ctx.synchronize()
    Qe = np.array(k["Q"], dtype=np.float64)
    assert np.abs(Q.cpu().numpy() - Qe).max() <= 1e-14 * max(np.abs(Qe).max(), 1.0), kat_id(k)
    for c, fe in enumerate(kat_expected_f(k, arrays)):
        assert np.abs(q[c].cpu().numpy() - fe).max() <= 1e-13 * np.abs(fe).max(), (kat_id(k), c)
