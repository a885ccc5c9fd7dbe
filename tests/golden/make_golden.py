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
