"""Generate tests/golden/kernel_weights.json -- known-answer 1-D weights.

The reference ships no tests or fixtures for this path and its
Fortran cannot be built here, so these vectors are computed independently of
the oracle: the reference's own 1-D delta-function formulas, evaluated in
60-digit decimal arithmetic at the stencil distances that the interaction
routines use:

* IB_4     -- lagrangian_ib_4_delta, lagrangian_delta.f.m4:209-233 (also
              ib4_kernel_fcn, LEInteractor.cpp:627-648)
* IB_4_W8  -- lagrangian_wide8_ib_4_delta = 0.5*ib4(r/2), lagrangian_delta.f.m4:240-252
* IB_3     -- lagrangian_ib_3_delta, lagrangian_delta.f.m4:158-180 (its truncated
              constants 0.16666666666667 / 0.333333333333333 kept)
* PIECEWISE_CUBIC -- lagrangian_piecewise_cubic_delta, lagrangian_delta.f.m4:109-130
* BSPLINE_4 -- cubic B-spline (not in the reference)
* IB_6     -- the 6-point kernel of the interaction routines (lagrangian_ib_6_
              interp3d, lagrangian_interaction3d.f.m4:1893, 1916-1945: K, the
              quadratic for pm3 with the sign(1, 3/2 - K) root and its linear
              combinations), transcribed here from the Fortran text, not from the
              C restatement.  (lagrangian_delta.f.m4:348's lagrangian_ib_6_delta
              is a different, older 6-point kernel that the interaction routines
              do not use.)  The script checks the defining moment conditions of
              the kernel in 60 digits before writing: sum 1, even/odd sums 1/2,
              first and third moments 0, second moment K.
* PIECEWISE_LINEAR -- the hat function lagrangian_piecewise_linear_delta
              (lagrangian_delta.f.m4:64-80) at the two points the routine picks
              (f.m4:636-658: the cell centre NINT(x - 1/2) + 1/2 and its neighbour
              on X's side)
* DISCONTINUOUS_LINEAR -- the hat function in the axis dim, the indicator of the
              cell NINT(x - 1/2) in the others (f.m4:258-282)
* PIECEWISE_CONSTANT -- the indicator of the cell NINT(x - 1/2) (f.m4:94-96)

Stencil placement per the interaction routines (ilower = 0):
  IB_4/BSPLINE_4: ic_lower = NINT(x) - 2 (lagrangian_interaction3d.f.m4:1317)
  IB_4_W8:        ic_lower = NINT(x) - 4 (:1595)
  IB_3 / PIECEWISE_CUBIC: floor-based centre (:1010-1040, :722-770)
and the weight of point j is phi(x - (j + 1/2)).

Run:  python tests/golden/make_golden.py   (rewrites kernel_weights.json)
"""
import json
from decimal import Decimal, getcontext
from pathlib import Path

getcontext().prec = 60
D = Decimal


def nint(x: Decimal) -> int:
    # Fortran NINT: nearest integer, halves away from zero (exact in Decimal)
    n = int((abs(x) + D("0.5")).to_integral_value(rounding="ROUND_FLOOR"))
    return n if x >= 0 else -n


def ffloor(x: Decimal) -> int:
    # lagrangian_floor: int(x) - (x < 0)
    f = int(x)
    return f - 1 if x < 0 else f


def ib4(r: Decimal) -> Decimal:
    r = abs(r)
    if r < 1:
        return -r / 4 + D(3) / 8 + (-4 * r * r + 4 * r + 1).sqrt() / 8
    if r < 2:
        return -r / 4 + D(5) / 8 - (12 * r - 7 - 4 * r * r).sqrt() / 8
    return D(0)


def bspline4(r: Decimal) -> Decimal:
    r = abs(r)
    if r < 1:
        return D(2) / 3 - r * r + r * r * r / 2
    if r < 2:
        return (2 - r) ** 3 / 6
    return D(0)


def ib3(r: Decimal) -> Decimal:
    sixth, third = D("0.16666666666667"), D("0.333333333333333")
    r = abs(r)
    if r < D("0.5"):
        return third * (1 + (1 - 3 * r * r).sqrt())
    if r < D("1.5"):
        return sixth * (5 - 3 * r - (1 - 3 * (1 - r) * (1 - r)).sqrt())
    return D(0)


def pwcubic(r: Decimal) -> Decimal:
    r = abs(r)
    if r < 1:
        return 1 - r / 2 - r * r + r * r * r / 2
    if r < 2:
        return 1 - D(11) / 6 * r + r * r - r * r * r / 6
    return D(0)


def ib6_K() -> Decimal:
    # f.m4:1893  K = (59/60) (1 - sqrt(1 - 3220/3481))
    return D(59) / 60 * (1 - (1 - D(3220) / 3481).sqrt())


def ib6_weights(x: Decimal, K: Decimal):
    # f.m4:1916-1945, term by term from the Fortran text
    icl = nint(x) - 3
    r = 1 - x + (D(icl + 2) + D("0.5"))
    alpha = D(28)
    beta = D(9) / 4 - D(3) / 2 * (K + r ** 2) + (D(22) / 3 - 7 * K) * r - D(7) / 3 * r ** 3
    gamma = D(1) / 4 * ((D(161) / 36 - D(59) / 6 * K + 5 * K ** 2) * D(1) / 2 * r ** 2
                        + (-D(109) / 24 + 5 * K) * D(1) / 3 * r ** 4 + D(5) / 18 * r ** 6)
    discr = beta ** 2 - 4 * alpha * gamma
    sgn = 1 if D(3) / 2 - K >= 0 else -1
    pm3 = (-beta + sgn * discr.sqrt()) / (2 * alpha)
    pm2 = -3 * pm3 - D(1) / 16 + D(1) / 8 * (K + r ** 2) + D(1) / 12 * (3 * K - 1) * r + D(1) / 12 * r ** 3
    pm1 = 2 * pm3 + D(1) / 4 + D(1) / 6 * (4 - 3 * K) * r - D(1) / 6 * r ** 3
    p0 = 2 * pm3 + D(5) / 8 - D(1) / 4 * (K + r ** 2)
    pp1 = -3 * pm3 + D(1) / 4 - D(1) / 6 * (4 - 3 * K) * r + D(1) / 6 * r ** 3
    pp2 = pm3 - D(1) / 16 + D(1) / 8 * (K + r ** 2) - D(1) / 12 * (3 * K - 1) * r - D(1) / 12 * r ** 3
    w = [pm3, pm2, pm1, p0, pp1, pp2]
    # the kernel's defining conditions (Bao, Kaiser, Peskin 2016), in 60 digits
    d = [x - (D(icl + j) + D("0.5")) for j in range(6)]
    tol = D("1e-45")
    assert abs(sum(w) - 1) < tol
    assert abs(w[0] + w[2] + w[4] - D("0.5")) < tol
    assert abs(sum(wj * dj for wj, dj in zip(w, d))) < tol
    assert abs(sum(wj * dj ** 2 for wj, dj in zip(w, d)) - K) < tol
    assert abs(sum(wj * dj ** 3 for wj, dj in zip(w, d))) < tol
    return icl, w


def hat(r: Decimal) -> Decimal:
    r = abs(r)
    return 1 - r if r < 1 else D(0)


XS = ["0.0", "0.25", "0.5", "0.75", "1.0", "2.5", "2.4999999999999996", "3.5000000000000004",
      "7.125", "-0.25", "-1.5", "-2.0", "5.3141592653589793", "12.999999999999998", "0.0001220703125"]


def main():
    out = {"source": __doc__.strip().splitlines()[0], "cases": []}
    for xs in XS:
        x = D(float(xs))  # the exact binary64 value the test feeds the oracle
        n = nint(x)
        # closed-form kernels
        for k, lo_off, W, phi, scale in (("IB_4", 2, 4, ib4, 1), ("BSPLINE_4", 2, 4, bspline4, 1),
                                         ("IB_4_W8", 4, 8, ib4, 2)):
            icl = n - lo_off
            w = []
            for j in range(W):
                dist = x - (D(icl + j) + D("0.5"))
                w.append(phi(dist / scale) / scale)
            out["cases"].append({"kernel": k, "X_o_dx": xs, "ic_lower": icl, "w": [str(v) for v in w]})
        K = ib6_K()
        icl6, w6 = ib6_weights(x, K)
        out["cases"].append({"kernel": "IB_6", "X_o_dx": xs, "ic_lower": icl6, "w": [str(v) for v in w6]})
        # low-order kernels: the cell NINT(x - 1/2), its centre, the side of x
        icc = nint(x - D("0.5"))
        xc = D(icc) + D("0.5")
        lo = icc - 1 if x < xc else icc
        out["cases"].append({"kernel": "PIECEWISE_LINEAR", "X_o_dx": xs, "ic_lower": lo,
                             "w": [str(hat(x - (D(j) + D("0.5")))) for j in (lo, lo + 1)]})
        out["cases"].append({"kernel": "DISCONTINUOUS_LINEAR", "X_o_dx": xs, "axis_dim": True, "ic_lower": lo,
                             "w": [str(hat(x - (D(j) + D("0.5")))) for j in (lo, lo + 1)]})
        out["cases"].append({"kernel": "DISCONTINUOUS_LINEAR", "X_o_dx": xs, "axis_dim": False, "ic_lower": icc,
                             "w": ["1"]})
        out["cases"].append({"kernel": "PIECEWISE_CONSTANT", "X_o_dx": xs, "ic_lower": icc, "w": ["1"]})
        # floor-centred kernels (point-wise delta evaluation)
        c = ffloor(x)
        xc = D(c) + D("0.5")
        for k, phi in (("IB_3", ib3), ("PIECEWISE_CUBIC", pwcubic)):
            if k == "IB_3":
                lo, hi = c - 1, c + 1
            else:
                lo, hi = (c - 2, c + 1) if x < xc else (c - 1, c + 2)
            w = [phi(x - (D(j) + D("0.5"))) for j in range(lo, hi + 1)]
            out["cases"].append({"kernel": k, "X_o_dx": xs, "ic_lower": lo, "w": [str(v) for v in w]})
    path = Path(__file__).with_name("kernel_weights.json")
    path.write_text(json.dumps(out, indent=1) + "\n")
    print(f"wrote {path} ({len(out['cases'])} cases)")


if __name__ == "__main__":
    main()
