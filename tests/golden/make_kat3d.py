"""Known-answer vectors for the 3-D side-centred IB_4 interp and spread, evaluated in
50-digit decimal arithmetic straight from the Fortran text -- independent of the
test oracle's C restatement (oracle/le_oracle.c) and of the device code.

Followed, line by line:
  * lagrangian_interaction3d.f.m4:1310-1382 (interp, IB_4) and :1447-1519 (spread):
    X_o_dx = (X + Xshift - x_lower)/dx, ic_lower = NINT(X_o_dx) + ilower - 2,
    r = X_o_dx - ((ic_lower + 1 - ilower) + 0.5), q = sqrt(1 + 4 r (1 - r)),
    w = ((3 - 2r - q), (3 - 2r + q), (1 + 2r + q), (1 + 2r - q)) / 8, the tensor
    product, the ghost-box clipping istart/istop, spread weights / (dx0 dx1 dx2);
  * LEInteractor.cpp:1017-1053 (interp) and :1876-1911 (spread) for SideData: per
    axis, x_lower[axis] -= dx[axis]/2 and the box is SideGeometry::toSideBox
    (iupper[axis] + 1); Q(s, axis) from the axis' pass (the last list entry naming
    a marker wins, as the Fortran's sequential loop).
NINT rounds halves away from zero (Fortran).  Inputs are dyadic (positions, dx,
x_lower, grid values), so every double operation before the square root is exact and
the decimal result is the true value of the Fortran formula; the tests hold double
results to it within 1e-13 (relative to the largest magnitude).

Markers: inside the patch, within the ghost region (stencils clipped by the ghost
box on low and high sides), and periodic images (Xshift = +-L), one marker listed
twice.  Run:  python tests/golden/make_kat3d.py  (writes kat3d_side_ib4.json).
"""
import json
import random
from decimal import Decimal, ROUND_HALF_UP, getcontext
from pathlib import Path

getcontext().prec = 50

ILOWER = [2, -1, 0]
IUPPER = [7, 3, 4]
GCW = 3
DX = [0.125, 0.25, 0.0625]
XLOWER = [ILOWER[d] * DX[d] for d in range(3)]
L = [(IUPPER[d] - ILOWER[d] + 1) * DX[d] for d in range(3)]


def side_box(axis):
    hi = list(IUPPER)
    hi[axis] += 1
    return list(ILOWER), hi


def shape_xyz(axis):
    lo, hi = side_box(axis)
    return [hi[d] - lo[d] + 1 + 2 * GCW for d in range(3)]


def nint(x):
    return int(x.quantize(Decimal(1), rounding=ROUND_HALF_UP))


def weights(X_o_dx, ilo):
    ic_lower = nint(X_o_dx) + ilo - 2
    r = X_o_dx - (Decimal(ic_lower + 1 - ilo) + Decimal("0.5"))
    q = (1 + 4 * r * (1 - r)).sqrt()
    w = [(3 - 2 * r - q) / 8, (3 - 2 * r + q) / 8, (1 + 2 * r + q) / 8, (1 + 2 * r - q) / 8]
    return ic_lower, w


def make():
    rng = random.Random(20261017)
    # grid values k/8, k in [-16, 16]: exact in double and decimal
    u = []
    for a in range(3):
        n = shape_xyz(a)
        u.append([[[rng.randint(-16, 16) / 8 for _ in range(n[0])] for _ in range(n[1])] for _ in range(n[2])])
    # markers: dyadic positions on a 1/64-cell lattice, away from NINT ties
    X = []
    for k in range(10):
        X.append([XLOWER[d] + (rng.randint(0, 64 * (IUPPER[d] - ILOWER[d] + 1) - 1) + 0.5) / 64 * DX[d]
                  for d in range(3)])
    # near the ghost box: a stencil of the x-axis pass reaching below ig_lower and
    # one of the z-axis pass beyond ig_upper
    X.append([XLOWER[0] - 2.75 * DX[0], XLOWER[1] + 1.5 / 64 * DX[1], XLOWER[2] + 3.25 * DX[2]])
    X.append([XLOWER[0] + 2.5 * DX[0] + DX[0] / 64, XLOWER[1] + (IUPPER[1] - ILOWER[1] + 1) * DX[1] + 2.4375 * DX[1],
              XLOWER[2] + (IUPPER[2] - ILOWER[2] + 1) * DX[2] + 2.625 * DX[2]])
    X.append([XLOWER[0] + 5.25 * DX[0], XLOWER[1] - 1.75 * DX[1], XLOWER[2] - 2.375 * DX[2]])
    M = len(X)
    F = [[rng.randint(-64, 64) / 16 for _ in range(3)] for _ in range(M)]
    # the list: every marker, two periodic images (Xshift = -+L in one or two dims),
    # marker 3 named again (the later entry's interp wins)
    indices = list(range(M)) + [0, 4, 3]
    Xshift = [[0.0, 0.0, 0.0] for _ in range(M)]
    Xshift.append([-L[0], 0.0, 0.0])
    Xshift.append([0.0, L[1], -L[2]])
    Xshift.append([0.0, 0.0, 0.0])
    # the images must still reach the ghost box: place markers 0 and 4 near the faces
    X[0] = [XLOWER[0] + L[0] - 0.625 * DX[0] + DX[0] / 128, X[0][1], X[0][2]]
    X[4] = [X[4][0], XLOWER[1] + 0.5 * DX[1] + DX[1] / 128, XLOWER[2] + L[2] - 0.75 * DX[2]]

    D = lambda v: Decimal(repr(float(v)))
    Q = [[None] * 3 for _ in range(M)]
    fout = []
    for a in range(3):
        lo, hi = side_box(a)
        ig_lo = [lo[d] - GCW for d in range(3)]
        ig_hi = [hi[d] + GCW for d in range(3)]
        xl = [D(XLOWER[d]) for d in range(3)]
        xl[a] -= D(DX[a]) / 2
        uarr = u[a]
        facc = [[[Decimal(0) for _ in row] for row in plane] for plane in uarr]
        for l, s in enumerate(indices):
            ic, w = [], []
            for d in range(3):
                c, wd = weights((D(X[s][d]) + D(Xshift[l][d]) - xl[d]) / D(DX[d]), lo[d])
                ic.append(c)
                w.append(wd)
            st = [max(ig_lo[d] - ic[d], 0) for d in range(3)]
            sp = [3 - max(ic[d] + 3 - ig_hi[d], 0) for d in range(3)]
            V = Decimal(0)
            h3 = D(DX[0]) * D(DX[1]) * D(DX[2])
            for i2 in range(st[2], sp[2] + 1):
                for i1 in range(st[1], sp[1] + 1):
                    for i0 in range(st[0], sp[0] + 1):
                        z, y, x = (ic[2] + i2 - ig_lo[2], ic[1] + i1 - ig_lo[1], ic[0] + i0 - ig_lo[0])
                        wt = w[0][i0] * w[1][i1] * w[2][i2]
                        V += wt * D(uarr[z][y][x])
                        facc[z][y][x] += wt / h3 * D(F[s][a])
            Q[s][a] = V
        fout.append([[[float(D(uarr[z][y][x]) + facc[z][y][x]) for x in range(len(uarr[0][0]))]
                      for y in range(len(uarr[0]))] for z in range(len(uarr))])
    return {
        "about": "3-D side-centred IB_4 interp/spread known answers, 50-digit decimal from the Fortran text "
                 "(tests/golden/make_kat3d.py)",
        "kernel": "IB_4", "ilower": ILOWER, "iupper": IUPPER, "gcw": GCW, "dx": DX, "x_lower": XLOWER,
        "u": u, "X": X, "F": F, "indices": indices, "Xshift": Xshift,
        "Q": [[float(v) for v in q] for q in Q], "f": fout,
    }


if __name__ == "__main__":
    out = Path(__file__).with_name("kat3d_side_ib4.json")
    out.write_text(json.dumps(make()))
    print("wrote", out)
