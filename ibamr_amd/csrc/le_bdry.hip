// le_bdry.hip -- physical-boundary ghost operators for side-centred data on one
// patch: the forward ghost fill (CartSideRobinPhysBdryOp::
// setPhysicalBoundaryConditions, CartSideRobinPhysBdryOp.cpp:358-422) that
// precedes interpolation, and its adjoint fold (accumulateFromPhysicalBoundary
// Data, :429-493) that LDataManager::spread runs after spreading
// (LDataManager.cpp:655-659).  The arithmetic is that of the Fortran routines
// in ibtk/src/boundary/physical_boundary/fortran/cartphysbdryop{2,3}d.f.m4.
//
// Work layout: one launch per boundary box (face, edge or corner) in the order
// the reference visits them.  Within a launch a thread owns a line of points
// that share every target of the accumulation (a tangential line of a face, an
// edge-parallel index, a side index of a corner) and walks the serial index in
// the Fortran's loop order, so every point receives its contributions in the
// reference's order: the result is bitwise the serial routine's.  The work is
// a few boundary planes, HBM-latency bound and small next to the sweeps.
#include <hip/hip_runtime.h>

#include "le_internal.h"

namespace ibtk_le {

namespace {

__device__ __forceinline__ double* at(const BdSide& P, int c, const int* x) {
    return P.u[c] + (x[0] - P.lo[c][0]) + (int64_t)(x[1] - P.lo[c][1]) * P.s1[c] +
           (int64_t)(x[2] - P.lo[c][2]) * P.s2[c];
}

// ghost cell range of direction d at the lower/upper end (the fill box)
__device__ __forceinline__ void ghost_range(const BdSide& P, int d, int upper, int& lo, int& hi) {
    lo = upper ? P.ihi[d] + 1 : P.ilo[d] - P.g;
    hi = upper ? P.ihi[d] + P.g : P.ilo[d] - 1;
}

// the tangential cell range of face normal n (extended by one along c when
// c >= 0, compute_tangential_extension, CartSideRobinPhysBdryOp.cpp:294-299);
// thread t -> point x on the face plane (x[n] left 0).  Returns false past the end.
__device__ __forceinline__ bool face_line(const BdSide& P, int n, int c, long t, int* x) {
    int ext[3] = {1, 1, 1};
    for (int d = 0; d < P.ndim; ++d)
        if (d != n) ext[d] = P.ihi[d] - P.ilo[d] + 1 + (d == c ? 1 : 0);
    if (t >= (long)ext[0] * ext[1] * ext[2]) return false;
    for (int d = 0; d < 3; ++d) {
        const int r = (int)(t % ext[d]);
        t /= ext[d];
        x[d] = d == n || d >= P.ndim ? 0 : P.ilo[d] + r;
    }
    return true;
}

}  // namespace

// scrobinphysbdryop1{x,y,z}{2,3}d (cartphysbdryop3d.f.m4:814-1185;
// 2d:396-629): the normal component of face loc; one thread per line.
__global__ __launch_bounds__(BLOCK) void k_bdry_sc1(BdSide P, int loc, double a, double b, double gv, int adjoint) {
    const int n = loc / 2, upper = loc & 1, g = P.g;
    int x[3];
    if (!face_line(P, n, -1, (long)blockIdx.x * BLOCK + threadIdx.x, x)) return;
    const double h = P.dx[loc / P.ndim];  // dx(location_index/NDIM), f.m4:872
    const int sgn = upper ? +1 : -1;
    const int i_b = upper ? P.ihi[n] + 1 : P.ilo[n];
    int xb[3] = {x[0], x[1], x[2]};
    xb[n] = i_b;
    double* const ub = at(P, n, xb);
    int xg[3] = {x[0], x[1], x[2]}, xi[3] = {x[0], x[1], x[2]};
    if (fabs(b) < 1.0e-12) {  // Dirichlet (f.m4:890-906)
        const double u_b = gv / a;
        *ub = u_b;
        for (int i = 1; i <= g; ++i) {
            xg[n] = i_b + sgn * i;
            xi[n] = i_b - sgn * i;
            if (adjoint) {
                const double u_g = *at(P, n, xg);
                double* const pi = at(P, n, xi);
                *pi = *pi + -1.0 * u_g;
                *ub = *ub + 2.0 * u_g;
            } else {
                *at(P, n, xg) = -1.0 * *at(P, n, xi) + 2.0 * u_b;
            }
        }
    } else {  // Robin (f.m4:907-925)
        const double u_b = *ub;
        for (int i = 1; i <= g; ++i) {
            const double nn = 2.0 * i;
            const double f_b = -(a * nn * h / b);
            const double f_g = nn * h / b;
            xg[n] = i_b + sgn * i;
            xi[n] = i_b - sgn * i;
            if (adjoint) {
                const double u_g = *at(P, n, xg);
                double* const pi = at(P, n, xi);
                *pi = *pi + 1.0 * u_g;
                *ub = *ub + f_b * u_g;
            } else {
                *at(P, n, xg) = 1.0 * *at(P, n, xi) + f_b * u_b + f_g * gv;
            }
        }
    }
}

// ccrobinphysbdryop1{x,y,z}{2,3}d (cartphysbdryop3d.f.m4:105-405; 2d:105-294)
// on the transverse components of face loc (CartSideRobinPhysBdryOp.cpp:
// 686-818): threads [0, n1) take component c1, the rest c2 (3-D).
__global__ __launch_bounds__(BLOCK) void k_bdry_cc1(BdSide P, int loc, int c1, int c2, long n1, BdCoef k1, BdCoef k2,
                                                    int adjoint) {
    const int n = loc / 2, upper = loc & 1, g = P.g;
    long t = (long)blockIdx.x * BLOCK + threadIdx.x;
    int c = c1;
    BdCoef k = k1;
    if (t >= n1) {
        if (c2 < 0) return;
        t -= n1;
        c = c2;
        k = k2;
    }
    int x[3];
    if (!face_line(P, n, c, t, x)) return;
    const double h = P.dx[loc / P.ndim];  // f.m4:162
    const int sgn = upper ? +1 : -1;
    const int i_g = upper ? P.ihi[n] + 1 : P.ilo[n] - 1;
    const int i_i = upper ? P.ihi[n] : P.ilo[n];
    int xg[3] = {x[0], x[1], x[2]}, xi[3] = {x[0], x[1], x[2]};
    for (int i = 0; i <= g - 1; ++i) {
        const double nn = 1.0 + 2.0 * i;
        const double f_i = -(k.a * nn * h - 2.0 * k.b) / (k.a * nn * h + 2.0 * k.b);
        const double f_g = 2.0 * nn * h / (k.a * nn * h + 2.0 * k.b);
        xg[n] = i_g + sgn * i;
        xi[n] = i_i - sgn * i;
        if (adjoint) {
            const double u_g = *at(P, c, xg);
            double* const pi = at(P, c, xi);
            *pi = *pi + f_i * u_g;
        } else {
            *at(P, c, xg) = f_i * *at(P, c, xi) + f_g * k.g;
        }
    }
}

// One codim-2 box: 3-D edge parallel to ea with normal directions p < q (or a
// 2-D corner, ea = -1, p = 0, q = 1).  Threads:
//   part 0: scrobinphysbdryop2 on component p, extrapolated along q
//           (one thread per (ea index, p side index), serial over q);
//   part 1: the same on component q along p;
//   part 2 (3-D): ccrobinphysbdryop23d on component ea (one thread per ea
//           side index, serial over q outer, p inner).
// cartphysbdryop3d.f.m4:1319-1478, 540-651; 2d:630-733.
__global__ __launch_bounds__(BLOCK) void k_bdry_edge(BdSide P, int ea, int p, int q, int up_p, int up_q, int adjoint) {
    long t = (long)blockIdx.x * BLOCK + threadIdx.x;
    const int g = P.g;
    const int nea = ea >= 0 ? P.ihi[ea] - P.ilo[ea] + 1 : 1;
    int up[3] = {0, 0, 0};
    up[p] = up_p;
    up[q] = up_q;
    for (int part = 0; part < 2; ++part) {
        const int c = part == 0 ? p : q, o = part == 0 ? q : p;
        const long cnt = (long)nea * g;
        if (t >= cnt) {
            t -= cnt;
            continue;
        }
        int x[3] = {0, 0, 0};
        if (ea >= 0) x[ea] = P.ilo[ea] + (int)(t % nea);
        int clo, chi;
        ghost_range(P, c, up[c], clo, chi);
        x[c] = clo + (up[c] ? 1 : 0) + (int)(t / nea);  // side ghost index along c
        int olo, ohi;
        ghost_range(P, o, up[o], olo, ohi);
        const int o_bdry = up[o] ? P.ihi[o] : P.ilo[o], o_shift = up[o] ? -1 : +1;
        int xb[3] = {x[0], x[1], x[2]}, xs[3] = {x[0], x[1], x[2]};
        xb[o] = o_bdry;
        xs[o] = o_bdry + o_shift;
        double* const pb = at(P, c, xb);
        double* const ps = at(P, c, xs);
        for (x[o] = olo; x[o] <= ohi; ++x[o]) {
            const double del = (double)abs(x[o] - o_bdry);
            if (adjoint) {
                const double u_g = *at(P, c, x);
                *pb = *pb + (1.0 + del) * u_g;
                *ps = *ps - del * u_g;
            } else {
                *at(P, c, x) = (1.0 + del) * *pb - del * *ps;
            }
        }
        return;
    }
    if (ea < 0 || t >= nea + 1) return;
    int x[3] = {0, 0, 0};
    x[ea] = P.ilo[ea] + (int)t;
    int plo, phi, qlo, qhi;
    ghost_range(P, p, up[p], plo, phi);
    ghost_range(P, q, up[q], qlo, qhi);
    const int p_bdry = up[p] ? P.ihi[p] : P.ilo[p], q_bdry = up[q] ? P.ihi[q] : P.ilo[q];
    const int sp = up[p] ? +1 : -1, sq = up[q] ? +1 : -1;
    for (x[q] = qlo; x[q] <= qhi; ++x[q]) {
        const int q_mirr = q_bdry + (q_bdry - x[q] + sq);
        for (x[p] = plo; x[p] <= phi; ++x[p]) {
            const int p_mirr = p_bdry + (p_bdry - x[p] + sp);
            int mm[3] = {x[0], x[1], x[2]}, bq[3] = {x[0], x[1], x[2]}, qb[3] = {x[0], x[1], x[2]};
            int bm[3] = {x[0], x[1], x[2]}, mb[3] = {x[0], x[1], x[2]};
            mm[p] = p_mirr, mm[q] = q_mirr;
            bq[p] = p_bdry;
            qb[q] = q_bdry;
            bm[p] = p_bdry, bm[q] = q_mirr;
            mb[p] = p_mirr, mb[q] = q_bdry;
            if (adjoint) {
                const double U_g = *at(P, ea, x);
                double* v;
                v = at(P, ea, mm), *v = *v + U_g;
                v = at(P, ea, bq), *v = *v + U_g;
                v = at(P, ea, qb), *v = *v + U_g;
                v = at(P, ea, bm), *v = *v - U_g;
                v = at(P, ea, mb), *v = *v - U_g;
            } else {
                *at(P, ea, x) = *at(P, ea, mm) + (*at(P, ea, bq) - *at(P, ea, bm)) + (*at(P, ea, qb) - *at(P, ea, mb));
            }
        }
    }
}

// scrobinphysbdryop33d (cartphysbdryop3d.f.m4:1480-1699), corner loc: thread
// (c, side ghost index along c), serial over o2 outer, o1 inner.
__global__ __launch_bounds__(64) void k_bdry_corner(BdSide P, int loc, int adjoint) {
    const int t = threadIdx.x, g = P.g;
    if (t >= 3 * g) return;
    const int c = t / g;
    const int up[3] = {loc & 1, (loc >> 1) & 1, (loc >> 2) & 1};
    const int o1 = c == 0 ? 1 : 0, o2 = c == 2 ? 1 : 2;
    int x[3];
    int clo, chi;
    ghost_range(P, c, up[c], clo, chi);
    x[c] = clo + (up[c] ? 1 : 0) + t % g;
    int lo1, hi1, lo2, hi2;
    ghost_range(P, o1, up[o1], lo1, hi1);
    ghost_range(P, o2, up[o2], lo2, hi2);
    const int b1 = up[o1] ? P.ihi[o1] : P.ilo[o1], s1 = up[o1] ? -1 : +1;
    const int b2 = up[o2] ? P.ihi[o2] : P.ilo[o2], s2 = up[o2] ? -1 : +1;
    int xbb[3] = {x[0], x[1], x[2]};
    xbb[o1] = b1, xbb[o2] = b2;
    int xsb[3] = {xbb[0], xbb[1], xbb[2]}, xbs[3] = {xbb[0], xbb[1], xbb[2]};
    xsb[o1] = b1 + s1;
    xbs[o2] = b2 + s2;
    double* const pbb = at(P, c, xbb);
    double* const psb = at(P, c, xsb);
    double* const pbs = at(P, c, xbs);
    for (x[o2] = lo2; x[o2] <= hi2; ++x[o2])
        for (x[o1] = lo1; x[o1] <= hi1; ++x[o1]) {
            const double d1 = (double)abs(x[o1] - b1), d2 = (double)abs(x[o2] - b2);
            if (adjoint) {
                const double u_g = *at(P, c, x);
                *pbb = *pbb + (1.0 + d1 + d2) * u_g;
                *psb = *psb - d1 * u_g;
                *pbs = *pbs - d2 * u_g;
            } else {
                *at(P, c, x) = (1.0 + d1 + d2) * *pbb - d1 * *psb - d2 * *pbs;
            }
        }
}

// ---------------------------------------------------------------------------
// host side: the boxes in the reference's order
// ---------------------------------------------------------------------------
static long face_lines(const BdSide& P, int n, int c) {
    long m = 1;
    for (int d = 0; d < P.ndim; ++d)
        if (d != n) m *= P.ihi[d] - P.ilo[d] + 1 + (d == c ? 1 : 0);
    return m;
}
static int blocks(long n) { return (int)((n + BLOCK - 1) / BLOCK); }

static hipError_t codim1_normal(const BdSide& P, const int* phys, const BdCoef* coef, int adjoint, hipStream_t s) {
    const int nf = 2 * P.ndim;
    for (int loc = 0; loc < nf; ++loc) {
        if (!phys[loc]) continue;
        const BdCoef k = coef[(loc / 2) * nf + loc];
        hipLaunchKernelGGL(k_bdry_sc1, dim3(blocks(face_lines(P, loc / 2, -1))), dim3(BLOCK), 0, s, P, loc, k.a, k.b,
                           k.g, adjoint);
    }
    return hipGetLastError();
}
static hipError_t codim1_transverse(const BdSide& P, const int* phys, const BdCoef* coef, int adjoint,
                                    hipStream_t s) {
    const int nf = 2 * P.ndim;
    for (int loc = 0; loc < nf; ++loc) {
        if (!phys[loc]) continue;
        const int n = loc / 2;
        int cs[2] = {-1, -1}, m = 0;
        for (int c = 0; c < P.ndim; ++c)
            if (c != n) cs[m++] = c;
        const long n1 = face_lines(P, n, cs[0]), n2 = cs[1] >= 0 ? face_lines(P, n, cs[1]) : 0;
        const BdCoef k1 = coef[cs[0] * nf + loc], k2 = cs[1] >= 0 ? coef[cs[1] * nf + loc] : k1;
        hipLaunchKernelGGL(k_bdry_cc1, dim3(blocks(n1 + n2)), dim3(BLOCK), 0, s, P, loc, cs[0], cs[1], n1, k1, k2,
                           adjoint);
    }
    return hipGetLastError();
}
static hipError_t codim2(const BdSide& P, const int* phys, int adjoint, hipStream_t s) {
    if (P.ndim == 2) {
        for (int loc = 0; loc < 4; ++loc) {
            const int ux = loc & 1, uy = (loc >> 1) & 1;
            if (!phys[ux] || !phys[2 + uy]) continue;
            hipLaunchKernelGGL(k_bdry_edge, dim3(blocks(2L * P.g)), dim3(BLOCK), 0, s, P, -1, 0, 1, ux, uy, adjoint);
        }
        return hipGetLastError();
    }
    for (int loc = 0; loc < 12; ++loc) {
        const int ea = loc / 4, n1 = (ea + 1) % 3, n2 = (ea + 2) % 3;  // cyclic order (SAMRAI)
        const int u1 = loc & 1, u2 = (loc >> 1) & 1;
        if (!phys[2 * n1 + u1] || !phys[2 * n2 + u2]) continue;
        const int p = n1 < n2 ? n1 : n2, q = n1 < n2 ? n2 : n1;
        const int up_p = p == n1 ? u1 : u2, up_q = q == n1 ? u1 : u2;
        const long nea = P.ihi[ea] - P.ilo[ea] + 1;
        hipLaunchKernelGGL(k_bdry_edge, dim3(blocks(2 * nea * P.g + nea + 1)), dim3(BLOCK), 0, s, P, ea, p, q, up_p,
                           up_q, adjoint);
    }
    return hipGetLastError();
}
static hipError_t codim3(const BdSide& P, const int* phys, int adjoint, hipStream_t s) {
    for (int loc = 0; loc < 8; ++loc) {
        if (!phys[loc & 1] || !phys[2 + ((loc >> 1) & 1)] || !phys[4 + ((loc >> 2) & 1)]) continue;
        hipLaunchKernelGGL(k_bdry_corner, dim3(1), dim3(64), 0, s, P, loc, adjoint);
    }
    return hipGetLastError();
}

hipError_t launch_phys_bdry_side(const BdSide& P, const int* phys, const BdCoef* coef, int adjoint, hipStream_t s) {
    hipError_t e;
    if (adjoint) {  // CartSideRobinPhysBdryOp.cpp:462-492
        if (P.ndim == 3 && (e = codim3(P, phys, 1, s)) != hipSuccess) return e;
        if ((e = codim2(P, phys, 1, s)) != hipSuccess) return e;
        if ((e = codim1_transverse(P, phys, coef, 1, s)) != hipSuccess) return e;
        return codim1_normal(P, phys, coef, 1, s);
    }
    // CartSideRobinPhysBdryOp.cpp:390-420
    if ((e = codim1_normal(P, phys, coef, 0, s)) != hipSuccess) return e;
    if ((e = codim1_transverse(P, phys, coef, 0, s)) != hipSuccess) return e;
    if ((e = codim2(P, phys, 0, s)) != hipSuccess) return e;
    if (P.ndim == 3) return codim3(P, phys, 0, s);
    return hipSuccess;
}

}  // namespace ibtk_le
