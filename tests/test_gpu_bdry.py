"""GPU: physical-boundary ghost fill and adjoint fold for side data
(ibtk_le_phys_bdry_side) against the oracle, bitwise.

CartSideRobinPhysBdryOp::setPhysicalBoundaryConditions (CartSideRobinPhysBdryOp.cpp:
358-422) and accumulateFromPhysicalBoundaryData (:429-493).  The device runs one
launch per boundary box in the reference's order and gives every target point its
contributions in the Fortran's loop order, so it must equal the serial oracle bit
for bit, for Dirichlet and Robin faces, inhomogeneous data, every face pattern.
"""
import zlib

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


CASES = [
    ([0, 0], [6, 5], 2),
    ([0, 0], [63, 63], 3),
    ([2, -1], [9, 6], 1),
    ([0, 0, 0], [5, 4, 6], 2),
    ([1, 0, -2], [6, 6, 3], 3),
    ([0, 0, 0], [47, 39, 31], 4),
]
PATTERNS = {
    "all": [1, 1, 1, 1, 1, 1],
    "walls_y": [0, 0, 1, 1, 0, 0],
    "mixed": [1, 0, 0, 1, 1, 1],
    "one": [0, 0, 0, 0, 0, 1],
}


def _coefs(rng, nd, kind):
    A = rng.uniform(0.5, 2.0, (nd, 2 * nd))
    B = rng.uniform(0.5, 2.0, (nd, 2 * nd))
    G = rng.uniform(-1.0, 1.0, (nd, 2 * nd))
    if kind == "dirichlet":
        B[:] = 0.0
    elif kind == "mixed":
        B[:, ::2] = 0.0  # lower faces Dirichlet, upper faces Robin
    return A, B, G


@pytest.mark.parametrize("lo,hi,g", CASES)
@pytest.mark.parametrize("pattern", list(PATTERNS))
@pytest.mark.parametrize("kind", ["robin", "dirichlet", "mixed"])
@pytest.mark.parametrize("adjoint", [True, False])
def test_phys_bdry_bitwise(le, ctx, lo, hi, g, pattern, kind, adjoint):
    nd = len(lo)
    rng = np.random.default_rng(zlib.crc32(repr((lo, hi, g, pattern, kind, adjoint)).encode()))
    phys = PATTERNS[pattern][:2 * nd]
    dx = [0.1, 0.13, 0.07][:nd]
    A, B, G = _coefs(rng, nd, kind)
    host = [rng.standard_normal(ora.side_ghost_shape(lo, hi, g, a)) for a in range(nd)]
    dev = [torch.from_numpy(h.copy()).cuda() for h in host]
    geom = le.Geometry(lo, hi, g, dx, [0.0] * nd)
    le.phys_bdry_side(ctx, geom, dev, phys, A, B, G, adjoint=adjoint)
    ctx.synchronize()
    ora.phys_bdry_side(lo, hi, g, dx, host, phys, A, B, G, adjoint=adjoint)
    for a in range(nd):
        got = dev[a].cpu().numpy()
        bad = np.argwhere(got.view(np.int64) != host[a].view(np.int64))
        assert bad.size == 0, f"comp {a}: {len(bad)} points differ, first {bad[:3].tolist()}"


def test_phys_bdry_rejects_bad_shapes(le, ctx):
    geom = le.Geometry([0, 0, 0], [7, 7, 7], 2, [0.1] * 3, [0.0] * 3)
    u = [torch.zeros(10, dtype=torch.float64, device="cuda") for _ in range(3)]
    with pytest.raises(ValueError):
        le.phys_bdry_side(ctx, geom, u, [1] * 6, 1.0, 1.0, 0.0, adjoint=True)


def test_phys_bdry_nonuniform_ghosts_error(le, ctx):
    geom = le.Geometry([0, 0, 0], [7, 7, 7], [2, 2, 3], [0.1] * 3, [0.0] * 3)
    u = [torch.zeros(geom.array_shape("side", a), dtype=torch.float64, device="cuda") for a in range(3)]
    with pytest.raises(Exception):
        le.phys_bdry_side(ctx, geom, u, [1] * 6, 1.0, 1.0, 0.0, adjoint=True)
