// le_stencil.h -- per-dimension stencil weights of the IBAMR kernel functions,
// device side.  Arithmetic is the Fortran's, operation by operation (see the
// citations), and is identical to the test oracle's C restatement so the two agree
// bit for bit when both are built with -ffp-contract=off.
#pragma once
#include <hip/hip_runtime.h>

#include "le_internal.h"

namespace ibtk_le {

// Kernel traits.  W = stencil points per dim; [LO, HI] bounds every stencil
// index of every centering frame relative to the key cell the marker is binned
// under (key = the family's cell-frame anchor, see key_anchor); FAM selects the
// arithmetic family.
//   FAM 0: closed-form weights on a NINT-anchored stencil, tensor product
//          w0*(w1*w2) (IB_4, IB_4_W8, IB_6, BSPLINE_4)
//   FAM 1: piecewise linear / discontinuous linear ((w0*w1)*w2)
//   FAM 2: pointwise delta evaluation after clipping (PIECEWISE_CUBIC, IB_3)
//   FAM 3: piecewise constant (single point)
template <int K> struct KT;
template <> struct KT<K_IB_4> { static constexpr int W = 4, LO = -2, HI = 2, FAM = 0; };
template <> struct KT<K_BSPLINE_4> { static constexpr int W = 4, LO = -2, HI = 2, FAM = 0; };
template <> struct KT<K_IB_6> { static constexpr int W = 6, LO = -3, HI = 3, FAM = 0; };
template <> struct KT<K_IB_4_W8> { static constexpr int W = 8, LO = -4, HI = 4, FAM = 0; };
template <> struct KT<K_PIECEWISE_LINEAR> { static constexpr int W = 2, LO = -1, HI = 2, FAM = 1; };
template <> struct KT<K_DISCONTINUOUS_LINEAR> { static constexpr int W = 2, LO = -1, HI = 2, FAM = 1; };
template <> struct KT<K_PIECEWISE_CUBIC> { static constexpr int W = 4, LO = -2, HI = 3, FAM = 2; };
template <> struct KT<K_IB_3> { static constexpr int W = 3, LO = -1, HI = 2, FAM = 2; };
template <> struct KT<K_PIECEWISE_CONSTANT> { static constexpr int W = 1, LO = 0, HI = 1, FAM = 3; };

#define IBTK_LE_CHECK_KT(K)                                                                       \
    static_assert(KT<K>::W == kKernelInfo[K].W && KT<K>::LO == kKernelInfo[K].LO && KT<K>::HI == kKernelInfo[K].HI, \
                  "kernel traits out of sync")
IBTK_LE_CHECK_KT(K_PIECEWISE_CONSTANT);
IBTK_LE_CHECK_KT(K_DISCONTINUOUS_LINEAR);
IBTK_LE_CHECK_KT(K_PIECEWISE_LINEAR);
IBTK_LE_CHECK_KT(K_PIECEWISE_CUBIC);
IBTK_LE_CHECK_KT(K_IB_3);
IBTK_LE_CHECK_KT(K_IB_4);
IBTK_LE_CHECK_KT(K_IB_4_W8);
IBTK_LE_CHECK_KT(K_IB_6);
IBTK_LE_CHECK_KT(K_BSPLINE_4);
#undef IBTK_LE_CHECK_KT

template <int W> struct St {
    int icl;       // index of weight 0
    int ist, isp;  // clipped weight range [ist, isp] (empty if ist > isp)
    double w[W];
};

// Fortran NINT (halves away from zero) -- llvm.round is exact.
__device__ __forceinline__ int d_nint(double x) { return (int)round(x); }
// lagrangian_floor, lagrangian_delta.f.m4:45-58
__device__ __forceinline__ int d_lfloor(double x) {
    int f = (int)x;
    if (x < 0.0) f = f - 1;
    return f;
}
// x**n by binary powering (same helper as the oracle)
__device__ __forceinline__ double d_powi(double x, int n) {
    double res = 1.0, cur = x;
    bool first = true;
    while (n) {
        if (n & 1) {
            res = first ? cur : res * cur;
            first = false;
        }
        n >>= 1;
        if (n) cur = cur * cur;
    }
    return res;
}

// lagrangian_piecewise_cubic_delta, lagrangian_delta.f.m4:109-130
__device__ __forceinline__ double d_pw_cubic_delta(double r) {
    if (r < 0.0) r = -r;
    if (r < 1.0) return 1.0 - 0.5 * r - r * r + 0.5 * r * r * r;
    if (r < 2.0) return 1.0 - (11.0 / 6.0) * r + r * r - (1.0 / 6.0) * r * r * r;
    return 0.0;
}
// lagrangian_ib_3_delta, lagrangian_delta.f.m4:158-180
__device__ __forceinline__ double d_ib3_delta(double r) {
    const double sixth = 0.16666666666667;
    const double third = 0.333333333333333;
    if (r < 0.0) r = -r;
    if (r < 0.5) return third * (1.0 + sqrt(1.0 - 3.0 * r * r));
    if (r < 1.5) return sixth * (5.0 - 3.0 * r - sqrt(1.0 - 3.0 * (1.0 - r) * (1.0 - r)));
    return 0.0;
}

// Key (bin) anchor of a marker in the cell frame: X_o_dx = (X+Xshift-x_lower)/dx.
template <int K> __device__ __forceinline__ int key_anchor(double X_o_dx) {
    constexpr int FAM = KT<K>::FAM;
    if constexpr (FAM == 0) return d_nint(X_o_dx);
    else if constexpr (FAM == 2) return d_lfloor(X_o_dx);
    else return d_nint(X_o_dx - 0.5);
}

// Closed-form 1-D weights; returns ic_lower.
//   IB_4:    lagrangian_interaction3d.f.m4:1316-1324
//   IB_4_W8: lagrangian_interaction3d.f.m4:1594-1610
//   IB_6:    lagrangian_interaction3d.f.m4:1914-1945
//   BSPLINE_4: cubic B-spline on the IB_4 stencil (not in the reference)
// sqrt(a) for a in [1, 2] (the IB_4 discriminant 1 + 4 r (1 - r), r in [0, 1]):
// the hardware reciprocal square root and two Newton steps, within an ulp of the
// correctly rounded root, no range scaling.  FAST closed weights only (the
// spread, compared by tolerance); the interp keeps sqrt() for bitwise parity.
__device__ __forceinline__ double sqrt_1_2(double a) {
    const double y = __builtin_amdgcn_rsq(a);
    double g = a * y, h = 0.5 * y;
    const double r = __builtin_fma(-g, h, 0.5);
    g = __builtin_fma(g, r, g);
    h = __builtin_fma(h, r, h);
    const double d = __builtin_fma(-g, g, a);
    return __builtin_fma(d, h, g);
}

template <int KID, bool FAST = false>
__device__ __forceinline__ int closed_weights(double X_o_dx, int ilower, double* w, double K6) {
    const int n = d_nint(X_o_dx);
    int ic_lower;
    if constexpr (KID == K_IB_4) {
        ic_lower = n + ilower - 2;
        const double r = X_o_dx - ((double)(ic_lower + 1 - ilower) + 0.5);
        const double q = FAST ? sqrt_1_2(1.0 + 4.0 * r * (1.0 - r)) : sqrt(1.0 + 4.0 * r * (1.0 - r));
        w[0] = 0.125 * (3.0 - 2.0 * r - q);
        w[1] = 0.125 * (3.0 - 2.0 * r + q);
        w[2] = 0.125 * (1.0 + 2.0 * r + q);
        w[3] = 0.125 * (1.0 + 2.0 * r - q);
    } else if constexpr (KID == K_BSPLINE_4) {
        ic_lower = n + ilower - 2;
        const double r = X_o_dx - ((double)(ic_lower + 1 - ilower) + 0.5);
        const double s = 1.0 - r;
        w[0] = (s * s * s) / 6.0;
        w[1] = (2.0 / 3.0) - r * r + 0.5 * (r * r * r);
        w[2] = (2.0 / 3.0) - s * s + 0.5 * (s * s * s);
        w[3] = (r * r * r) / 6.0;
    } else if constexpr (KID == K_IB_4_W8) {
        ic_lower = n + ilower - 4;
        double r = 0.5 * (X_o_dx - ((double)(ic_lower + 3 - ilower) + 0.5));
        double q = sqrt(1.0 + 4.0 * r * (1.0 - r));
        w[1] = 0.0625 * (3.0 - 2.0 * r - q);
        w[3] = 0.0625 * (3.0 - 2.0 * r + q);
        w[5] = 0.0625 * (1.0 + 2.0 * r + q);
        w[7] = 0.0625 * (1.0 + 2.0 * r - q);
        r = r + 0.5;
        q = sqrt(1.0 + 4.0 * r * (1.0 - r));
        w[0] = 0.0625 * (3.0 - 2.0 * r - q);
        w[2] = 0.0625 * (3.0 - 2.0 * r + q);
        w[4] = 0.0625 * (1.0 + 2.0 * r + q);
        w[6] = 0.0625 * (1.0 + 2.0 * r - q);
    } else {  // IB_6
        const double K = K6;
        ic_lower = n + ilower - 3;
        const double r = 1.0 - X_o_dx + ((double)(ic_lower + 2 - ilower) + 0.5);
        const double r2 = d_powi(r, 2), r3 = d_powi(r, 3), r4 = d_powi(r, 4), r6 = d_powi(r, 6);
        const double alpha = 28.0;
        const double beta = (9.0 / 4.0) - (3.0 / 2.0) * (K + r2) + ((22.0 / 3.0) - 7.0 * K) * r - (7.0 / 3.0) * r3;
        const double gamma = (1.0 / 4.0) * (((161.0 / 36.0) - (59.0 / 6.0) * K + 5.0 * d_powi(K, 2)) * (1.0 / 2.0) * r2 +
                                             (-(109.0 / 24.0) + 5.0 * K) * (1.0 / 3.0) * r4 + (5.0 / 18.0) * r6);
        const double discr = beta * beta - 4.0 * alpha * gamma;
        const double sgn = ((3.0 / 2.0) - K) >= 0.0 ? 1.0 : -1.0;
        const double pm3 = (-beta + sgn * sqrt(discr)) / (2.0 * alpha);
        w[0] = pm3;
        w[1] = -3.0 * pm3 - (1.0 / 16.0) + (1.0 / 8.0) * (K + r2) + (1.0 / 12.0) * (3.0 * K - 1.0) * r +
               (1.0 / 12.0) * r3;
        w[2] = 2.0 * pm3 + (1.0 / 4.0) + (1.0 / 6.0) * (4.0 - 3.0 * K) * r - (1.0 / 6.0) * r3;
        w[3] = 2.0 * pm3 + (5.0 / 8.0) - (1.0 / 4.0) * (K + r2);
        w[4] = -3.0 * pm3 + (1.0 / 4.0) - (1.0 / 6.0) * (4.0 - 3.0 * K) * r + (1.0 / 6.0) * r3;
        w[5] = pm3 - (1.0 / 16.0) + (1.0 / 8.0) * (K + r2) - (1.0 / 12.0) * (3.0 * K - 1.0) * r - (1.0 / 12.0) * r3;
    }
    return ic_lower;
}

// One dimension of one component's stencil: weights + clipped range.
//   Xs   = X(d,s) + Xshift(d,l);  Xraw = X(d,s)
//   xlo  = the component frame's x_lower(d);  ilo = its ilower(d)
//   [glo, ghi] = the component array's ghost box in dim d
//   axis_dim = (d == axis) for DISCONTINUOUS_LINEAR
//   MUL: X_o_dx by a multiply with inv_dx = 1/dx instead of the Fortran's
//        division (closed-form kernels only): within an ulp of it, for the
//        spread, whose sums are compared by tolerance, not bit for bit
#ifndef IBTK_LE_FAST_SQRT
#define IBTK_LE_FAST_SQRT 1
#endif
template <int K, bool MUL = false>
__device__ __forceinline__ void stencil1d(double Xs, double Xraw, double xlo, double dx, int ilo, int glo, int ghi,
                                          bool axis_dim, double K6, St<KT<K>::W>& st, double inv_dx = 0.0) {
    constexpr int W = KT<K>::W;
    constexpr int FAM = KT<K>::FAM;
    if constexpr (FAM == 0) {
        // f.m4:1316 (X_o_dx), :1360-1365 (istart/istop)
        // MUL: near a NINT tie the product can round to the other side of it than
        // the quotient (which the bin key uses), moving the stencil one cell.
        // At a tie the end weight of these kernels is 0 (r = 0 or 1), so the
        // point that may then fall outside the key's bands carries a weight of
        // an ulp's order: within the spread's tolerance.
        const double X_o_dx = MUL ? (Xs - xlo) * inv_dx : (Xs - xlo) / dx;
        st.icl = closed_weights<K, MUL && IBTK_LE_FAST_SQRT>(X_o_dx, ilo, st.w, K6);
        const int icu = st.icl + (W - 1);
        st.ist = max(glo - st.icl, 0);
        st.isp = (W - 1) - max(icu - ghi, 0);
    } else if constexpr (FAM == 1) {
        // pw-linear f.m4:636-658 / disc-linear f.m4:258-282
        const int icc = ilo + d_nint((Xs - xlo) / dx - 0.5);
        const double Xc = xlo + ((double)(icc - ilo) + 0.5) * dx;
        int lo, up;
        if (K == K_PIECEWISE_LINEAR || axis_dim) {
            if (Xs < Xc) {
                lo = icc - 1;
                up = icc;
                st.w[0] = (Xc - Xs) / dx;
                st.w[1] = 1.0 - st.w[0];
            } else {
                lo = icc;
                up = icc + 1;
                st.w[0] = 1.0 + (Xc - Xs) / dx;
                st.w[1] = 1.0 - st.w[0];
            }
        } else {
            st.w[0] = 1.0;
            st.w[1] = 0.0;
            lo = icc;
            up = icc;
        }
        st.icl = lo;
        st.ist = max(lo, glo) - lo;
        st.isp = min(up, ghi) - lo;
    } else if constexpr (FAM == 2) {
        // pw-cubic f.m4:722-791 (side decided with the UNSHIFTED X), IB_3 f.m4:1006-1050
        const int icc = d_lfloor((Xs - xlo) / dx) + ilo;
        const double Xc = xlo + ((double)(icc - ilo) + 0.5) * dx;
        int lo, up;
        if constexpr (K == K_PIECEWISE_CUBIC) {
            if (Xraw < Xc) {
                lo = icc - 2;
                up = icc + 1;
            } else {
                lo = icc - 1;
                up = icc + 2;
            }
        } else {
            lo = icc - 1;
            up = icc + 1;
        }
        lo = max(lo, glo);
        up = min(up, ghi);
        st.icl = lo;
        st.ist = 0;
        st.isp = up - lo;
#pragma unroll
        for (int j = 0; j < W; ++j) {
            const int ic = lo + j;
            const double Xci = xlo + ((double)(ic - ilo) + 0.5) * dx;
            const double r = (Xs - Xci) / dx;
            st.w[j] = (j <= st.isp) ? (K == K_PIECEWISE_CUBIC ? d_pw_cubic_delta(r) : d_ib3_delta(r)) : 0.0;
        }
    } else {
        // piecewise constant f.m4:100-103.  The reference does not clip; an
        // out-of-box cell is treated as an empty stencil here.
        const int ic = d_nint((Xs - xlo) / dx - 0.5) + ilo;
        st.icl = ic;
        st.w[0] = 1.0;
        st.ist = 0;
        st.isp = (ic >= glo && ic <= ghi) ? 0 : -1;
    }
}

}  // namespace ibtk_le
