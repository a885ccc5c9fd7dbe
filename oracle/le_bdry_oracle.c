/*
 * le_bdry_oracle.c -- CPU restatement of IBTK's physical-boundary operators for
 * side-centred data (TEST INFRASTRUCTURE ONLY).
 *
 * Only tests/ may load this (through oracle/oracle.py), as the checker of the
 * device implementation in ibamr_amd/csrc/le_bdry.hip.  The product library
 * never links, calls or falls back to it.
 *
 * PARITY STATUS: "parity unpinned" against the reference binary, for the same
 * reason as le_oracle.c: the reference routines are m4 sources
 * (ibtk/src/boundary/physical_boundary/fortran/cartphysbdryop{2,3}d.f.m4) that
 * need the absent m4 processor and SAMRAI's unvendored array-dimension macros,
 * and the reference ships no tests or recorded outputs for them.  The
 * restatement is pinned by identities instead (tests/test_oracle_bdry.py):
 * the adjoint routine is the transpose of the forward one wherever the Fortran
 * makes it so (Robin faces, extrapolated edges and corners), the forward fill
 * reproduces linear data along every extrapolation, and hand-worked values.
 *
 * What is restated:
 *   CartSideRobinPhysBdryOp::setPhysicalBoundaryConditions
 *     (CartSideRobinPhysBdryOp.cpp:358-422) -- adjoint = 0, and
 *   CartSideRobinPhysBdryOp::accumulateFromPhysicalBoundaryData
 *     (CartSideRobinPhysBdryOp.cpp:429-493) -- adjoint = 1,
 * for one patch whose faces flagged in `phys` lie on a non-periodic physical
 * boundary, with Robin coefficients a, b, g constant over each face
 * (RobinBcCoefStrategy::setBcCoefs filling a constant box; index NDIM*d + axis
 * with depth d = 0, CartSideRobinPhysBdryOp.cpp:545-546).  SAMRAI's boundary
 * boxes of such a patch (PhysicalBoundaryUtilities::getPhysicalBoundaryCodim
 * {1,2,3}Boxes, PatchGeometry::getBoundaryFillBox) are restated as: a codim-1
 * box per physical face spanning the patch in the tangential directions, a
 * codim-2 box per edge (3-D) / corner (2-D) whose two faces are both physical,
 * a codim-3 box per corner whose three faces are; each fill box is `g` cells
 * deep in its normal directions.  Location indices follow SAMRAI: faces
 * 2 d + upper; 3-D edges 4 a + bit0 + 2 bit1 with the two normal directions in
 * cyclic order after the edge axis a (cartphysbdryop3d.f.m4:1245-1317);
 * corners bit0 = upper x, bit1 = upper y, bit2 = upper z.
 *
 * Reference quirks restated as they are:
 *   - h = dx(location_index/NDIM) (cartphysbdryop3d.f.m4:162, 872): in 3-D the
 *     y-lower face takes dx(0) and the z faces dx(1);
 *   - a Dirichlet face (|b| < 1e-12) overwrites the boundary value with g/a
 *     before accumulating in the adjoint too (cartphysbdryop3d.f.m4:890-899).
 *
 * Every loop nest runs in the Fortran's order, so every point receives its
 * contributions in the reference's order.  Compile with -ffp-contract=off.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>

#include "le_oracle.h"

typedef struct {
    int ndim, g;
    int ilo[3], ihi[3];
    double dx[3];
    double* u[3];
    int lo[3][3];           /* ghost-box lower corner of component c */
    int64_t s1[3], s2[3];   /* strides of component c */
} bd_patch;

static inline double* U(const bd_patch* P, int c, int i, int j, int k)
{
    return P->u[c] + (i - P->lo[c][0]) + (int64_t)(j - P->lo[c][1]) * P->s1[c] +
           (int64_t)(k - P->lo[c][2]) * P->s2[c];
}

/* point (x0, x1, x2) of component c */
static inline double* Uv(const bd_patch* P, int c, const int* x) { return U(P, c, x[0], x[1], x[2]); }

/* ccrobinphysbdryop1{x,y,z}3d (cartphysbdryop3d.f.m4:105-405; 2d:105-294):
 * the transverse component c on face loc, lines over bc_coef_box = the face's
 * tangential cell range extended by one along c (compute_tangential_extension,
 * CartSideRobinPhysBdryOp.cpp:693-694). */
static void ora_cc1(const bd_patch* P, int c, int loc, double a, double b, double gv, int adjoint)
{
    const int nd = P->ndim, g = P->g, n = loc / 2;
    const double h = P->dx[loc / nd];
    const int sgn = (loc % 2) ? +1 : -1;
    const int i_g = (loc % 2) ? P->ihi[n] + 1 : P->ilo[n] - 1;
    const int i_i = (loc % 2) ? P->ihi[n] : P->ilo[n];
    int blo[3] = {0, 0, 0}, bhi[3] = {0, 0, 0};
    for (int d = 0; d < nd; ++d) {
        blo[d] = P->ilo[d];
        bhi[d] = P->ihi[d] + (d == c ? 1 : 0);
    }
    blo[n] = bhi[n] = 0;
    int x[3];
    for (int t2 = blo[2]; t2 <= bhi[2]; ++t2)
        for (int t1 = blo[1]; t1 <= bhi[1]; ++t1)
            for (int t0 = blo[0]; t0 <= bhi[0]; ++t0) {
                x[0] = t0, x[1] = t1, x[2] = t2;
                for (int i = 0; i <= g - 1; ++i) {
                    const double nn = 1.0 + 2.0 * i;
                    const double f_i = -(a * nn * h - 2.0 * b) / (a * nn * h + 2.0 * b);
                    const double f_g = 2.0 * nn * h / (a * nn * h + 2.0 * b);
                    int xg[3] = {x[0], x[1], x[2]}, xi[3] = {x[0], x[1], x[2]};
                    xg[n] = i_g + sgn * i;
                    xi[n] = i_i - sgn * i;
                    if (adjoint) {
                        const double u_g = *Uv(P, c, xg);
                        *Uv(P, c, xi) = *Uv(P, c, xi) + f_i * u_g;
                    } else {
                        const double u_i = *Uv(P, c, xi);
                        *Uv(P, c, xg) = f_i * u_i + f_g * gv;
                    }
                }
            }
}

/* scrobinphysbdryop1{x,y,z}3d (cartphysbdryop3d.f.m4:814-1185; 2d:396-629):
 * the normal component on face loc, lines over the tangential cell range. */
static void ora_sc1(const bd_patch* P, int loc, double a, double b, double gv, int adjoint)
{
    const int nd = P->ndim, g = P->g, n = loc / 2;
    const double h = P->dx[loc / nd];
    const int sgn = (loc % 2) ? +1 : -1;
    const int i_b = (loc % 2) ? P->ihi[n] + 1 : P->ilo[n];
    int blo[3] = {0, 0, 0}, bhi[3] = {0, 0, 0};
    for (int d = 0; d < nd; ++d) {
        blo[d] = P->ilo[d];
        bhi[d] = P->ihi[d];
    }
    blo[n] = bhi[n] = 0;
    int x[3];
    for (int t2 = blo[2]; t2 <= bhi[2]; ++t2)
        for (int t1 = blo[1]; t1 <= bhi[1]; ++t1)
            for (int t0 = blo[0]; t0 <= bhi[0]; ++t0) {
                x[0] = t0, x[1] = t1, x[2] = t2;
                int xb[3] = {x[0], x[1], x[2]};
                xb[n] = i_b;
                double* const ub = Uv(P, n, xb);
                if (fabs(b) < 1.0e-12) {  /* Dirichlet */
                    const double u_b = gv / a;
                    *ub = u_b;
                    for (int i = 1; i <= g; ++i) {
                        const double f_i = -1.0, f_b = 2.0;
                        int xg[3] = {x[0], x[1], x[2]}, xi[3] = {x[0], x[1], x[2]};
                        xg[n] = i_b + sgn * i;
                        xi[n] = i_b - sgn * i;
                        if (adjoint) {
                            const double u_g = *Uv(P, n, xg);
                            *Uv(P, n, xi) = *Uv(P, n, xi) + f_i * u_g;
                            *ub = *ub + f_b * u_g;
                        } else {
                            const double u_i = *Uv(P, n, xi);
                            *Uv(P, n, xg) = f_i * u_i + f_b * u_b;
                        }
                    }
                } else {  /* Robin */
                    const double u_b = *ub;
                    for (int i = 1; i <= g; ++i) {
                        const double nn = 2.0 * i;
                        const double f_i = 1.0;
                        const double f_b = -a * nn * h / b;
                        const double f_g = nn * h / b;
                        int xg[3] = {x[0], x[1], x[2]}, xi[3] = {x[0], x[1], x[2]};
                        xg[n] = i_b + sgn * i;
                        xi[n] = i_b - sgn * i;
                        if (adjoint) {
                            const double u_g = *Uv(P, n, xg);
                            *Uv(P, n, xi) = *Uv(P, n, xi) + f_i * u_g;
                            *ub = *ub + f_b * u_g;
                        } else {
                            const double u_i = *Uv(P, n, xi);
                            *Uv(P, n, xg) = f_i * u_i + f_b * u_b + f_g * gv;
                        }
                    }
                }
            }
}

/* boundary index and inward shift of direction d at the lower/upper end */
static inline void bdry_of(const bd_patch* P, int d, int upper, int* bd, int* shift)
{
    *bd = upper ? P->ihi[d] : P->ilo[d];
    *shift = upper ? -1 : +1;
}
/* ghost cell range of direction d at the lower/upper end (fill box) */
static inline void ghost_range(const bd_patch* P, int d, int upper, int* lo, int* hi)
{
    *lo = upper ? P->ihi[d] + 1 : P->ilo[d] - P->g;
    *hi = upper ? P->ihi[d] + P->g : P->ilo[d] - 1;
}

/* One component loop of scrobinphysbdryop2{2,3}d (cartphysbdryop3d.f.m4:
 * 1319-1478; 2d:630-733): component c (a normal direction of the edge) over
 * its side-index ghost range along c, extrapolated along the other normal
 * direction o; along the edge axis ea (3-D) the patch's cell range.
 * Loop order: dims 2, 1, 0 outer to inner, as every Fortran nest here. */
static void ora_sc2_comp(const bd_patch* P, int c, int o, int ea, const int* up, int adjoint)
{
    int blo[3] = {0, 0, 0}, bhi[3] = {0, 0, 0};
    ghost_range(P, c, up[c], &blo[c], &bhi[c]);
    if (up[c]) ++blo[c], ++bhi[c];  /* side indices beyond the upper face: ihi+2 .. ihi+g+1 */
    ghost_range(P, o, up[o], &blo[o], &bhi[o]);
    if (ea >= 0) blo[ea] = P->ilo[ea], bhi[ea] = P->ihi[ea];
    int o_bdry, o_shift;
    bdry_of(P, o, up[o], &o_bdry, &o_shift);
    int x[3];
    for (x[2] = blo[2]; x[2] <= bhi[2]; ++x[2])
        for (x[1] = blo[1]; x[1] <= bhi[1]; ++x[1])
            for (x[0] = blo[0]; x[0] <= bhi[0]; ++x[0]) {
                const double del = (double)abs(x[o] - o_bdry);
                int xb[3] = {x[0], x[1], x[2]}, xs[3] = {x[0], x[1], x[2]};
                xb[o] = o_bdry;
                xs[o] = o_bdry + o_shift;
                if (adjoint) {
                    const double u_g = *Uv(P, c, x);
                    *Uv(P, c, xb) = *Uv(P, c, xb) + (1.0 + del) * u_g;
                    *Uv(P, c, xs) = *Uv(P, c, xs) - del * u_g;
                } else {
                    *Uv(P, c, x) = (1.0 + del) * *Uv(P, c, xb) - del * *Uv(P, c, xs);
                }
            }
}

/* ccrobinphysbdryop23d (cartphysbdryop3d.f.m4:408-651): the edge-parallel
 * component ea over toSideBox(fill box, ea) (CartSideRobinPhysBdryOp.cpp:
 * 884-902), mirrored linear extrapolation in the two normal directions p < q. */
static void ora_cc2(const bd_patch* P, int ea, int p, int q, const int* up, int adjoint)
{
    int blo[3] = {0, 0, 0}, bhi[3] = {0, 0, 0};
    blo[ea] = P->ilo[ea], bhi[ea] = P->ihi[ea] + 1;
    ghost_range(P, p, up[p], &blo[p], &bhi[p]);
    ghost_range(P, q, up[q], &blo[q], &bhi[q]);
    const int p_bdry = up[p] ? P->ihi[p] : P->ilo[p], q_bdry = up[q] ? P->ihi[q] : P->ilo[q];
    const int sp = up[p] ? +1 : -1, sq = up[q] ? +1 : -1;
    int x[3];
    for (x[2] = blo[2]; x[2] <= bhi[2]; ++x[2])
        for (x[1] = blo[1]; x[1] <= bhi[1]; ++x[1])
            for (x[0] = blo[0]; x[0] <= bhi[0]; ++x[0]) {
                const int p_mirr = p_bdry + (p_bdry - x[p] + sp), q_mirr = q_bdry + (q_bdry - x[q] + sq);
                int mm[3] = {x[0], x[1], x[2]}, bq[3] = {x[0], x[1], x[2]}, qb[3] = {x[0], x[1], x[2]};
                int bm[3] = {x[0], x[1], x[2]}, mb[3] = {x[0], x[1], x[2]};
                mm[p] = p_mirr, mm[q] = q_mirr;  /* U(i, j_mirr, k_mirr) */
                bq[p] = p_bdry;                  /* U(i, j_bdry, k)      */
                qb[q] = q_bdry;                  /* U(i, j, k_bdry)      */
                bm[p] = p_bdry, bm[q] = q_mirr;  /* U(i, j_bdry, k_mirr) */
                mb[p] = p_mirr, mb[q] = q_bdry;  /* U(i, j_mirr, k_bdry) */
                if (adjoint) {
                    const double U_g = *Uv(P, ea, x);
                    *Uv(P, ea, mm) = *Uv(P, ea, mm) + U_g;
                    *Uv(P, ea, bq) = *Uv(P, ea, bq) + U_g;
                    *Uv(P, ea, qb) = *Uv(P, ea, qb) + U_g;
                    *Uv(P, ea, bm) = *Uv(P, ea, bm) - U_g;
                    *Uv(P, ea, mb) = *Uv(P, ea, mb) - U_g;
                } else {
                    *Uv(P, ea, x) = *Uv(P, ea, mm) + (*Uv(P, ea, bq) - *Uv(P, ea, bm)) +
                                    (*Uv(P, ea, qb) - *Uv(P, ea, mb));
                }
            }
}

/* One component loop of scrobinphysbdryop33d (cartphysbdryop3d.f.m4:1480-1699):
 * component c over its side-index ghost range, extrapolated along the two other
 * directions o1 < o2. */
static void ora_sc3_comp(const bd_patch* P, int c, const int* up, int adjoint)
{
    const int o1 = c == 0 ? 1 : 0, o2 = c == 2 ? 1 : 2;
    int blo[3], bhi[3];
    for (int d = 0; d < 3; ++d) ghost_range(P, d, up[d], &blo[d], &bhi[d]);
    if (up[c]) ++blo[c], ++bhi[c];
    int b1, s1, b2, s2;
    bdry_of(P, o1, up[o1], &b1, &s1);
    bdry_of(P, o2, up[o2], &b2, &s2);
    int x[3];
    for (x[2] = blo[2]; x[2] <= bhi[2]; ++x[2])
        for (x[1] = blo[1]; x[1] <= bhi[1]; ++x[1])
            for (x[0] = blo[0]; x[0] <= bhi[0]; ++x[0]) {
                const double d1 = (double)abs(x[o1] - b1), d2 = (double)abs(x[o2] - b2);
                int xbb[3] = {x[0], x[1], x[2]}, xsb[3], xbs[3];
                xbb[o1] = b1, xbb[o2] = b2;
                xsb[0] = xbb[0], xsb[1] = xbb[1], xsb[2] = xbb[2];
                xbs[0] = xbb[0], xbs[1] = xbb[1], xbs[2] = xbb[2];
                xsb[o1] = b1 + s1;
                xbs[o2] = b2 + s2;
                if (adjoint) {
                    const double u_g = *Uv(P, c, x);
                    *Uv(P, c, xbb) = *Uv(P, c, xbb) + (1.0 + d1 + d2) * u_g;
                    *Uv(P, c, xsb) = *Uv(P, c, xsb) - d1 * u_g;
                    *Uv(P, c, xbs) = *Uv(P, c, xbs) - d2 * u_g;
                } else {
                    *Uv(P, c, x) = (1.0 + d1 + d2) * *Uv(P, c, xbb) - d1 * *Uv(P, c, xsb) - d2 * *Uv(P, c, xbs);
                }
            }
}

static void ora_codim3(const bd_patch* P, const int* phys, int adjoint)
{
    for (int loc = 0; loc < 8; ++loc) {
        const int up[3] = {loc & 1, (loc >> 1) & 1, (loc >> 2) & 1};
        if (!phys[up[0]] || !phys[2 + up[1]] || !phys[4 + up[2]]) continue;
        for (int c = 0; c < 3; ++c) ora_sc3_comp(P, c, up, adjoint);
    }
}

static void ora_codim2(const bd_patch* P, const int* phys, int adjoint)
{
    if (P->ndim == 2) {
        for (int loc = 0; loc < 4; ++loc) {
            const int up[3] = {loc & 1, (loc >> 1) & 1, 0};
            if (!phys[up[0]] || !phys[2 + up[1]]) continue;
            ora_sc2_comp(P, 0, 1, -1, up, adjoint);  /* u0 along y (2d:703-716) */
            ora_sc2_comp(P, 1, 0, -1, up, adjoint);  /* u1 along x (2d:717-731) */
        }
        return;
    }
    for (int loc = 0; loc < 12; ++loc) {
        const int ea = loc / 4;
        const int n1 = (ea + 1) % 3, n2 = (ea + 2) % 3;  /* cyclic order */
        int up[3] = {0, 0, 0};
        up[n1] = loc & 1;
        up[n2] = (loc >> 1) & 1;
        if (!phys[2 * n1 + up[n1]] || !phys[2 * n2 + up[n2]]) continue;
        const int p = n1 < n2 ? n1 : n2, q = n1 < n2 ? n2 : n1;
        /* scrobinphysbdryop23d: component p extrapolated along q, then q along p */
        ora_sc2_comp(P, p, q, ea, up, adjoint);
        ora_sc2_comp(P, q, p, ea, up, adjoint);
        ora_cc2(P, ea, p, q, up, adjoint);
    }
}

static void ora_codim1_transverse(const bd_patch* P, const int* phys, const double* A, const double* B,
                                  const double* G, int adjoint)
{
    const int nd = P->ndim;
    for (int loc = 0; loc < 2 * nd; ++loc) {
        if (!phys[loc]) continue;
        for (int c = 0; c < nd; ++c) {
            if (c == loc / 2) continue;
            const int k = c * 2 * nd + loc;
            ora_cc1(P, c, loc, A[k], B[k], G[k], adjoint);
        }
    }
}

static void ora_codim1_normal(const bd_patch* P, const int* phys, const double* A, const double* B, const double* G,
                              int adjoint)
{
    const int nd = P->ndim;
    for (int loc = 0; loc < 2 * nd; ++loc) {
        if (!phys[loc]) continue;
        const int k = (loc / 2) * 2 * nd + loc;
        ora_sc1(P, loc, A[k], B[k], G[k], adjoint);
    }
}

int ora_phys_bdry_side(int ndim, const int* ilower, const int* iupper, int gcw, const double* dx, double* u0,
                       double* u1, double* u2, const int* phys, const double* acoef, const double* bcoef,
                       const double* gcoef, int adjoint)
{
    if (ndim != 2 && ndim != 3) return 1;
    if (gcw <= 0) return 0;  /* ghost_width_to_fill == 0: nothing to do */
    bd_patch P;
    P.ndim = ndim;
    P.g = gcw;
    double* us[3] = {u0, u1, u2};
    for (int d = 0; d < 3; ++d) {
        P.ilo[d] = d < ndim ? ilower[d] : 0;
        P.ihi[d] = d < ndim ? iupper[d] : 0;
        P.dx[d] = d < ndim ? dx[d] : 0.0;
        P.u[d] = d < ndim ? us[d] : 0;
    }
    for (int c = 0; c < ndim; ++c) {
        int64_t n[3] = {1, 1, 1};
        for (int d = 0; d < 3; ++d) {
            const int g = d < ndim ? gcw : 0;
            P.lo[c][d] = P.ilo[d] - g;
            n[d] = (P.ihi[d] + g + (d == c ? 1 : 0)) - P.lo[c][d] + 1;
        }
        P.s1[c] = n[0];
        P.s2[c] = n[0] * n[1];
    }
    if (adjoint) {  /* CartSideRobinPhysBdryOp.cpp:462-492 */
        if (ndim == 3) ora_codim3(&P, phys, 1);
        ora_codim2(&P, phys, 1);
        ora_codim1_transverse(&P, phys, acoef, bcoef, gcoef, 1);
        ora_codim1_normal(&P, phys, acoef, bcoef, gcoef, 1);
    } else {        /* CartSideRobinPhysBdryOp.cpp:390-420 */
        ora_codim1_normal(&P, phys, acoef, bcoef, gcoef, 0);
        ora_codim1_transverse(&P, phys, acoef, bcoef, gcoef, 0);
        ora_codim2(&P, phys, 0);
        if (ndim == 3) ora_codim3(&P, phys, 0);
    }
    return 0;
}
