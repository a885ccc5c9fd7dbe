"""GPU: size-independent properties at BASELINE.json's full sizes (cfg4: 1024^3
periodic staggered grid, 1e8 uniform markers, IB_4; cfg3: 512^3, 1e7, IB_6 and
BSPLINE_4), where
the oracle would take hours.

* conservation: sum over the unique grid points of S F times h^3 equals sum F, per
  component (the kernels' partition of unity);
* adjointness: <J u, F> over the markers equals h^3 <u, S F> over the unique points
  (interp and spread are transposes, LEInteractor.cpp's shared stencils);
* interpolating a constant field returns the constant;
* spreading is bit-stable run to run at full size.
The sums run in fp64 over 1e8-1e9 terms; the tolerances (1e-10 relative) bound
their rounding, not the kernels'.
"""
import pytest

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


def _unique(t, g, N):
    return t[g:g + N, g:g + N, g:g + N]


@pytest.mark.parametrize("N,M,kernel", [(256, 2_000_000, "IB_4"), (512, 10_000_000, "IB_6"),
                                        (512, 10_000_000, "BSPLINE_4"), (1024, 100_000_000, "IB_4")])
def test_fullsize_properties(le, ctx, N, M, kernel):
    g = le._lib.load().ibtk_le_min_ghost_width(le.kernel_id(kernel))
    geom = le.Geometry.periodic_unit([N] * 3, ghost=g)
    h3 = geom.dx[0] * geom.dx[1] * geom.dx[2]
    gen = torch.Generator(device="cuda").manual_seed(1234)
    X = torch.rand((M, 3), dtype=torch.float64, device="cuda", generator=gen)
    F = torch.rand((M, 3), dtype=torch.float64, device="cuda", generator=gen) * 2 - 1
    m = le.Markers(ctx).bin(geom, kernel, X)
    # spread + fold, twice (bit stability)
    f = geom.alloc("side")
    le.spread(ctx, m, kernel, "side", geom, f, F, X)
    le.fold_periodic_ghosts(ctx, geom, "side", f)
    f2 = [torch.zeros_like(t) for t in f]
    le.spread(ctx, m, kernel, "side", geom, f2, F, X)
    le.fold_periodic_ghosts(ctx, geom, "side", f2)
    ctx.synchronize()
    for a in range(3):
        assert torch.equal(f[a], f2[a]), f"component {a} not bit-stable"
    del f2
    # conservation
    for a in range(3):
        tot = _unique(f[a], g, N).sum().item() * h3
        ref = F[:, a].sum().item()
        assert abs(tot - ref) <= 1e-10 * F[:, a].abs().sum().item(), (a, tot, ref)
    # adjointness with a random periodic field
    u = geom.alloc("side")
    for t in u:
        t.uniform_(-1, 1, generator=gen)
    le.fill_periodic_ghosts(ctx, geom, "side", u)
    Q = torch.zeros((M, 3), dtype=torch.float64, device="cuda")
    le.interp(ctx, m, kernel, "side", geom, u, Q, X)
    ctx.synchronize()
    lhs = (Q * F).sum().item()
    rhs = h3 * sum((_unique(u[a], g, N) * _unique(f[a], g, N)).sum().item() for a in range(3))
    scale = (Q.abs() * F.abs()).sum().item()
    assert abs(lhs - rhs) <= 1e-10 * scale, (lhs, rhs)
    # constant field
    for t in u:
        t.fill_(0.75)
    le.interp(ctx, m, kernel, "side", geom, u, Q, X)
    ctx.synchronize()
    assert (Q - 0.75).abs().max().item() <= 1e-14
