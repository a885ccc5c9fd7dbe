// le_hot.hip -- the hot path on CDNA4 (gfx950): marker binning, interpolation
// and spreading.  Replaces the l-loops of
// ibtk/src/lagrangian/fortran/lagrangian_interaction{2,3}d.f.m4.
//
// Work decomposition:
//  * bin: key = brick id (tiled, le_bricks.h) << 9 | cell-in-brick of the
//    marker's cell-frame stencil anchor; stable device radix sort; brick CSR;
//    then one coalescing pass writes the sorted marker index and the sorted
//    shifted position X(s)+Xshift(l), so the interp/spread kernels read their
//    markers contiguously.
//  * interp: one workgroup item = (brick, component).  The union stencil region
//    of the brick's markers, (8+HI-LO)^3 points of that component, is loaded
//    from HBM with every load of a thread in flight at once and staged in LDS
//    (13.8 KB for IB_4, so ~11 items are resident per CU); one thread per marker
//    then sums its W^3 stencil from LDS in the Fortran loop order, so the result
//    is bitwise the oracle's.
//  * spread: one workgroup item = (super-brick of 16^3 cells, component).  The
//    workgroup loads u_old of its 4096 points into LDS, walks the sorted entries
//    of the 4x4x4 surrounding bricks in canonical (sorted) order, keeps those
//    whose stencil can reach the super-brick (parallel filter + ordered block
//    compaction), computes their 1-D weights in parallel, and one wave then adds
//    candidate after candidate with lane = stencil point (ds_add_f64 into LDS).
//    Each grid point therefore receives its contributions in list order exactly
//    like the Fortran's sequential l-loop: no global atomics, deterministic,
//    bitwise the oracle's on the same list.  16^3 super-bricks keep the halo
//    over-processing at (20/16)^3 = 1.95x the owned markers for IB_4.
#include <hip/hip_runtime.h>

#include <climits>
#include <cstdlib>

#include "le_bricks.h"
#include "le_internal.h"
#include "le_stencil.h"

namespace ibtk_le {

constexpr int IBLOCK = 128;  // interp workgroup (2 waves)
constexpr int SBLOCK = 256;  // spread workgroup (4 waves)

static int num_cus() {
    static int ncu = 0;
    if (!ncu) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0)
            ncu = 256;
    }
    return ncu;
}

static int grid_for(long items, int per_cu) {
    long g = (long)num_cus() * per_cu;
    if (g > items) g = items;
    if (g >= 8) g &= ~7L;
    return (int)(g > 0 ? g : 1);
}

// ---------------------------------------------------------------------------
// binning
// ---------------------------------------------------------------------------
template <int NDIM, int K>
__global__ __launch_bounds__(BLOCK) void k_bin(Params p, int n, unsigned* keys, int* vals) {
    constexpr int B = BrickT<NDIM>::B;
    const int i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n) return;
    const int s = p.indices ? p.indices[i] : i;
    bool out = false;
    int rel[3] = {0, 0, 0};
#pragma unroll
    for (int d = 0; d < NDIM; ++d) {
        const double Xs = p.X[(int64_t)NDIM * s + d] + (p.Xshift ? p.Xshift[(int64_t)NDIM * i + d] : 0.0);
        const double xo = (Xs - p.bg.xlo[d]) / p.bg.dx[d];
        if (!(fabs(xo) < 1.0e9)) {  // also catches NaN
            out = true;
            continue;
        }
        rel[d] = key_anchor<K>(xo) + p.bg.ilower[d] - p.bg.kmin[d];
        if (rel[d] < 0 || rel[d] >= p.bg.nb[d] * B) out = true;
    }
    unsigned key;
    if (out) {
        key = (unsigned)p.bg.nbricks << BrickT<NDIM>::SHIFT;
    } else {
        int bc[3] = {0, 0, 0};
        unsigned local = 0;
        for (int d = NDIM - 1; d >= 0; --d) {
            bc[d] = rel[d] / B;
            local = local * (unsigned)B + (unsigned)(rel[d] - bc[d] * B);
        }
        key = ((unsigned)brick_id<NDIM>(p.bg, bc) << BrickT<NDIM>::SHIFT) | local;
    }
    keys[i] = key;
    vals[i] = i;
}

// brick_start[b] = first sorted position whose bucket >= b, for b in [0, nbricks].
__global__ __launch_bounds__(BLOCK) void k_brick_start(const unsigned* keys, int n, int nbricks, int shift, int* bs) {
    const int i = blockIdx.x * BLOCK + threadIdx.x;
    if (i > n) return;
    const int bi = (i < n) ? (int)min(keys[i] >> shift, (unsigned)nbricks) : nbricks + 1;
    const int bp = (i == 0) ? -1 : (int)min(keys[i - 1] >> shift, (unsigned)nbricks);
    for (int b = bp + 1; b <= bi && b <= nbricks; ++b) bs[b] = i;
}

// sorted marker index and sorted X(s) + Xshift(l) (the Fortran's X(d,s)+Xshift(d,l))
template <int NDIM>
__global__ __launch_bounds__(BLOCK) void k_gather_sorted(Params p, int n, int* sorted_s, double* sorted_X) {
    const int e = blockIdx.x * BLOCK + threadIdx.x;
    if (e >= n) return;
    const int l = p.sorted_l[e];
    const int s = p.indices ? p.indices[l] : l;
    sorted_s[e] = s;
#pragma unroll
    for (int d = 0; d < NDIM; ++d)
        sorted_X[(int64_t)NDIM * e + d] =
            p.X[(int64_t)NDIM * s + d] + (p.Xshift ? p.Xshift[(int64_t)NDIM * l + d] : 0.0);
}

template <int NDIM, int K>
hipError_t launch_bin_t(const Params& p, int n, unsigned* keys, int* vals, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL((k_bin<NDIM, K>), dim3((n + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, s, p, n, keys, vals);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// interpolation
// ---------------------------------------------------------------------------
template <int NDIM, int K> struct IShape {
    using T = KT<K>;
    static constexpr int B = BrickT<NDIM>::B;
    static constexpr int R = B + T::HI - T::LO;  // region edge (points)
    static constexpr int RV = NDIM == 3 ? R * R * R : R * R;
    static constexpr int NL = (RV + IBLOCK - 1) / IBLOCK;  // staged values per thread
};

template <int NDIM, int K>
__device__ __forceinline__ void marker_stencils_x(const Params& p, const CompDesc& cd, const double* Xs, int s,
                                                  St<KT<K>::W>* st) {
    constexpr int FAM = KT<K>::FAM;
#pragma unroll
    for (int d = 0; d < NDIM; ++d) {
        const double Xraw = (FAM == 2) ? p.X[(int64_t)NDIM * s + d] : Xs[d];
        stencil1d<K>(Xs[d], Xraw, cd.xlo[d], p.bg.dx[d], cd.ilower[d], cd.lo[d], cd.hi[d], d == cd.axis, p.K6,
                     st[d]);
    }
}

template <int NDIM, int K>
__device__ __forceinline__ void marker_stencils(const Params& p, const CompDesc& cd, int e, int s,
                                                St<KT<K>::W>* st) {
    double Xs[NDIM];
#pragma unroll
    for (int d = 0; d < NDIM; ++d) Xs[d] = p.sorted_X[(int64_t)NDIM * e + d];
    marker_stencils_x<NDIM, K>(p, cd, Xs, s, st);
}

template <int NDIM, int K>
__global__ __launch_bounds__(IBLOCK) void k_interp(Params p) {
    using T = KT<K>;
    using S = IShape<NDIM, K>;
    constexpr int W = T::W, FAM = T::FAM, B = S::B, R = S::R, RV = S::RV, NL = S::NL;
    extern __shared__ __attribute__((aligned(16))) double reg[];
    const int nc = p.ncomp;
    const int nitems = p.bg.nbricks * nc;
    const int G = gridDim.x;
    for (int round = 0; round < nitems; round += G) {
        const int it = xcd_item(round, G, blockIdx.x);
        if (it >= nitems) continue;
        const int b = it / nc, c = it - (it / nc) * nc;
        const int beg = p.brick_start[b], end = p.brick_start[b + 1];
        if (beg == end) continue;
        int bc[3];
        brick_coords<NDIM>(p.bg, b, bc);
        int r0[3] = {0, 0, 0};
        bool inside = true;
        const CompDesc& cd = p.comp[c];
#pragma unroll
        for (int d = 0; d < NDIM; ++d) {
            r0[d] = p.bg.kmin[d] + bc[d] * B + T::LO;
            inside = inside && r0[d] >= cd.lo[d] && r0[d] + R - 1 <= cd.hi[d];
        }
        // this thread's first marker, loaded together with the staging loads
        const int e0 = beg + threadIdx.x;
        int s0 = 0;
        double x0[NDIM];
        if (e0 < end) {
            s0 = p.sorted_s[e0];
#pragma unroll
            for (int d = 0; d < NDIM; ++d) x0[d] = p.sorted_X[(int64_t)NDIM * e0 + d];
        }
        // issue every staging load of this thread before using any of them
        double v[NL];
        const int64_t o0 = (int64_t)(r0[0] - cd.lo[0]) + (int64_t)(r0[1] - cd.lo[1]) * cd.s1 +
                           (NDIM == 3 ? (int64_t)(r0[2] - cd.lo[2]) * cd.s2 : 0);
#pragma unroll
        for (int k = 0; k < NL; ++k) {
            const int q = threadIdx.x + k * IBLOCK;
            v[k] = 0.0;
            if (q < RV) {
                const int i0 = q % R, i1 = (q / R) % R, i2 = NDIM == 3 ? q / (R * R) : 0;
                if (inside) {
                    v[k] = cd.u[o0 + i0 + (int64_t)i1 * cd.s1 + (NDIM == 3 ? (int64_t)i2 * cd.s2 : 0)];
                } else {
                    const int g0 = r0[0] + i0, g1 = r0[1] + i1, g2 = r0[2] + i2;
                    bool in = g0 >= cd.lo[0] && g0 <= cd.hi[0] && g1 >= cd.lo[1] && g1 <= cd.hi[1];
                    if (NDIM == 3) in = in && g2 >= cd.lo[2] && g2 <= cd.hi[2];
                    if (in)
                        v[k] = cd.u[(int64_t)(g0 - cd.lo[0]) + (int64_t)(g1 - cd.lo[1]) * cd.s1 +
                                    (NDIM == 3 ? (int64_t)(g2 - cd.lo[2]) * cd.s2 : 0)];
                }
            }
        }
        __syncthreads();  // the previous item's readers are done with reg
#pragma unroll
        for (int k = 0; k < NL; ++k) {
            const int q = threadIdx.x + k * IBLOCK;
            if (q < RV) reg[q] = v[k];
        }
        __syncthreads();

        for (int e = e0; e < end; e += IBLOCK) {
            int s = s0;
            if (e != e0) {
                s = p.sorted_s[e];
#pragma unroll
                for (int d = 0; d < NDIM; ++d) x0[d] = p.sorted_X[(int64_t)NDIM * e + d];
            }
            St<W> st[NDIM];
            marker_stencils_x<NDIM, K>(p, cd, x0, s, st);
            bool ok = true;
#pragma unroll
            for (int d = 0; d < NDIM; ++d)
                if (st[d].ist <= st[d].isp)
                    ok = ok && (st[d].icl + st[d].ist >= r0[d]) && (st[d].icl + st[d].isp < r0[d] + R);
            if (!ok) {
                atomicOr(p.err, 1);
                continue;
            }
            double acc = 0.0;
            if constexpr (FAM == 3) {
                bool nonempty = true;
#pragma unroll
                for (int d = 0; d < NDIM; ++d) nonempty = nonempty && (st[d].ist <= st[d].isp);
                if (nonempty) {
                    int li = st[0].icl - r0[0] + R * (st[1].icl - r0[1]);
                    if (NDIM == 3) li += R * R * (st[2].icl - r0[2]);
                    acc = reg[li];
                }
            } else {
                // Clipped stencil entries (outside [ist, isp]) get weight 0 and a
                // clamped (in-region) LDS index: acc + 0 == acc, so the sum equals
                // the Fortran's clipped sum bit for bit, without per-term branches.
                double w[NDIM][W];
                int o[NDIM][W];
#pragma unroll
                for (int d = 0; d < NDIM; ++d) {
                    const int stride = d == 0 ? 1 : (d == 1 ? R : R * R);
#pragma unroll
                    for (int i = 0; i < W; ++i) {
                        const bool in = i >= st[d].ist && i <= st[d].isp;
                        w[d][i] = in ? st[d].w[i] : 0.0;
                        o[d][i] = min(max(st[d].icl + i - r0[d], 0), R - 1) * stride;
                    }
                }
                if constexpr (NDIM == 3) {
#pragma unroll
                    for (int i2 = 0; i2 < W; ++i2) {
#pragma unroll
                        for (int i1 = 0; i1 < W; ++i1) {
                            const double* row = reg + o[1][i1] + o[2][i2];
                            if constexpr (FAM == 0) {
                                const double wyz = w[1][i1] * w[2][i2];  // f.m4:1349-1353
#pragma unroll
                                for (int i0 = 0; i0 < W; ++i0) {
                                    const double wt = w[0][i0] * wyz;
                                    acc = acc + wt * row[o[0][i0]];  // f.m4:1375
                                }
                            } else {
#pragma unroll
                                for (int i0 = 0; i0 < W; ++i0)
                                    acc = acc + w[0][i0] * w[1][i1] * w[2][i2] * row[o[0][i0]];  // f.m4:545-548
                            }
                        }
                    }
                } else {
#pragma unroll
                    for (int i1 = 0; i1 < W; ++i1) {
                        const double* row = reg + o[1][i1];
#pragma unroll
                        for (int i0 = 0; i0 < W; ++i0) {
                            if constexpr (FAM == 0) {
                                const double wt = w[0][i0] * w[1][i1];
                                acc = acc + wt * row[o[0][i0]];
                            } else {
                                acc = acc + w[0][i0] * w[1][i1] * row[o[0][i0]];
                            }
                        }
                    }
                }
            }
            p.Qout[(int64_t)p.Q_depth * s + cd.qcomp] = acc;
        }
    }
}

// Entries binned "outside" (no stencil point can reach any array): V = 0.
__global__ __launch_bounds__(BLOCK) void k_interp_outside(Params p, int n) {
    const int first = p.brick_start[p.bg.nbricks];
    for (int e = first + blockIdx.x * BLOCK + threadIdx.x; e < n; e += gridDim.x * BLOCK) {
        const int s = p.sorted_s[e];
        for (int c = 0; c < p.ncomp; ++c) p.Qout[(int64_t)p.Q_depth * s + p.comp[c].qcomp] = 0.0;
    }
}

// Direct form: one thread per sorted entry, every component, stencil values read
// straight from HBM/L2 (no staging).  Neighbouring threads hold neighbouring
// markers, so a wave's loads hit a compact set of lines.  Entries binned
// "outside" get V = 0 (their clipped stencil is empty).
template <int NDIM, int K>
__global__ __launch_bounds__(BLOCK) void k_interp_direct(Params p, int n) {
    using T = KT<K>;
    constexpr int W = T::W, FAM = T::FAM;
    const int blk = xcd_item(0, gridDim.x, blockIdx.x);
    const int e = blk * BLOCK + threadIdx.x;
    if (e >= n) return;
    const unsigned key = p.sorted_key[e];
    const int s = p.sorted_s[e];
    double Xs[NDIM];
#pragma unroll
    for (int d = 0; d < NDIM; ++d) Xs[d] = p.sorted_X[(int64_t)NDIM * e + d];
    const bool out = (key >> BrickT<NDIM>::SHIFT) >= (unsigned)p.bg.nbricks;
    for (int c = 0; c < p.ncomp; ++c) {
        const CompDesc& cd = p.comp[c];
        double acc = 0.0;
        if (!out) {
            St<W> st[NDIM];
            marker_stencils_x<NDIM, K>(p, cd, Xs, s, st);
            if constexpr (FAM == 3) {
                bool nonempty = true;
#pragma unroll
                for (int d = 0; d < NDIM; ++d) nonempty = nonempty && (st[d].ist <= st[d].isp);
                if (nonempty)
                    acc = cd.u[(int64_t)(st[0].icl - cd.lo[0]) + (int64_t)(st[1].icl - cd.lo[1]) * cd.s1 +
                               (NDIM == 3 ? (int64_t)(st[2 % NDIM].icl - cd.lo[2]) * cd.s2 : 0)];
            } else {
                // clipped entries: weight 0 at a clamped (in-array) index, acc + 0 == acc
                double w[NDIM][W];
                int64_t o[NDIM][W];
#pragma unroll
                for (int d = 0; d < NDIM; ++d) {
                    const int64_t stride = d == 0 ? 1 : (d == 1 ? cd.s1 : cd.s2);
#pragma unroll
                    for (int i = 0; i < W; ++i) {
                        const bool in = i >= st[d].ist && i <= st[d].isp;
                        w[d][i] = in ? st[d].w[i] : 0.0;
                        o[d][i] = (int64_t)(min(max(st[d].icl + i, cd.lo[d]), cd.hi[d]) - cd.lo[d]) * stride;
                    }
                }
                if constexpr (NDIM == 3) {
#pragma unroll
                    for (int i2 = 0; i2 < W; ++i2) {
#pragma unroll
                        for (int i1 = 0; i1 < W; ++i1) {
                            const double* row = cd.u + o[1][i1] + o[2][i2];
                            if constexpr (FAM == 0) {
                                const double wyz = w[1][i1] * w[2][i2];  // f.m4:1349-1353
#pragma unroll
                                for (int i0 = 0; i0 < W; ++i0) {
                                    const double wt = w[0][i0] * wyz;
                                    acc = acc + wt * row[o[0][i0]];  // f.m4:1375
                                }
                            } else {
#pragma unroll
                                for (int i0 = 0; i0 < W; ++i0)
                                    acc = acc + w[0][i0] * w[1][i1] * w[2][i2] * row[o[0][i0]];  // f.m4:545-548
                            }
                        }
                    }
                } else {
#pragma unroll
                    for (int i1 = 0; i1 < W; ++i1) {
                        const double* row = cd.u + o[1][i1];
#pragma unroll
                        for (int i0 = 0; i0 < W; ++i0) {
                            if constexpr (FAM == 0) {
                                const double wt = w[0][i0] * w[1][i1];
                                acc = acc + wt * row[o[0][i0]];
                            } else {
                                acc = acc + w[0][i0] * w[1][i1] * row[o[0][i0]];
                            }
                        }
                    }
                }
            }
        }
        p.Qout[(int64_t)p.Q_depth * s + cd.qcomp] = acc;
    }
}

static int interp_mode() {
    static int mode = -1;
    if (mode < 0) {
        const char* v = getenv("IBTK_LE_INTERP");
        mode = (v && v[0] == 's') ? 0 : 1;  // 0 staged, 1 direct
    }
    return mode;
}

template <int NDIM, int K>
hipError_t launch_interp_t(const Params& p, int n, hipStream_t s, hipEvent_t ev0, hipEvent_t ev1) {
    using S = IShape<NDIM, K>;
    const size_t lds = (size_t)S::RV * sizeof(double);
    if (lds > 64 * 1024)
        (void)hipFuncSetAttribute((const void*)k_interp<NDIM, K>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)lds);
    if (ev0) (void)hipEventRecord(ev0, s);
    if (interp_mode() == 1) {
        if (n > 0) hipLaunchKernelGGL((k_interp_direct<NDIM, K>), dim3((n + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, s, p, n);
        if (ev1) (void)hipEventRecord(ev1, s);
        return hipGetLastError();
    }
    const long items = (long)p.bg.nbricks * p.ncomp;
    hipLaunchKernelGGL((k_interp<NDIM, K>), dim3(grid_for(items, 16)), dim3(IBLOCK), lds, s, p);
    if (ev1) (void)hipEventRecord(ev1, s);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    if (n > 0) hipLaunchKernelGGL(k_interp_outside, dim3(64), dim3(BLOCK), 0, s, p, n);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// spreading
// ---------------------------------------------------------------------------
template <int NDIM, int K> struct SShape {
    using BT = BrickT<NDIM>;
    static constexpr int B = BT::B, SB = BT::SB, SBV = BT::SBV, GROUP = BT::GROUP;
    static constexpr int W = KT<K>::W;
    static constexpr int P = NDIM == 3 ? W * W * W : W * W;  // stencil points
    static constexpr int NPASS = (P + 63) / 64;              // 64-lane passes per stencil
    static constexpr int NQ = SBLOCK / 64;                   // waves = quarters of the super-brick
    static constexpr int QW = SB / NQ;                       // planes (3-D z) / rows (2-D y) per quarter
    static constexpr int NBR = NDIM == 3 ? 64 : 16;          // neighbourhood bricks (4 per dim)
    static constexpr int KMAX = 2;                           // entries per thread per filter pass
    static constexpr int CAP = KMAX * SBLOCK;                // candidates per filter pass
    static constexpr int CH = W <= 4 ? 128 : 64;             // candidates per prep/process chunk
    static constexpr int NWD = CH / 64;                      // 64-bit words of a chunk bitmap
    static constexpr int RWD = NDIM * W + 1;                 // record doubles: 1-D weights, F
    static constexpr int NACC = SBV / SBLOCK;                // u values per thread
    static constexpr int LB = NDIM == 3 ? 3 : 4;             // log2(B)
};

// sorted_F[c * n + e] = Q(qcomp_c, s(e)): the spread values in sorted order, so
// the spread kernel's loads of them are contiguous and not behind the s load.
__global__ __launch_bounds__(BLOCK) void k_gather_F(Params p, int n, double* out) {
    const int e = blockIdx.x * BLOCK + threadIdx.x;
    if (e >= n) return;
    const int s = p.sorted_s[e];
    for (int c = 0; c < p.ncomp; ++c)
        out[(int64_t)c * n + e] = p.Qin[(int64_t)p.Q_depth * s + p.comp[c].qcomp];
}

// One workgroup item = one super-brick (16^3 cells in 3-D, 32^2 in 2-D), all
// components in turn.  Per component the super-brick's u_old goes to LDS; the
// entries of the surrounding 4^NDIM bricks are walked in canonical (sorted)
// order and those whose stencil can reach the super-brick kept (parallel
// filter + ordered compaction, done once for all components when they fit one
// pass); chunks of candidates get their stencils computed one per thread into
// LDS records, with a bitmap per quarter (a quarter = QW planes along the last
// dim, owned by one wave) of the candidates that touch it.  Each wave then walks
// its bitmap in ascending order -- the scalar unit finds the next set bit, so a
// wave never visits a candidate that misses its quarter -- adding the candidate's
// stencil points (lane = stencil point) with ds_add_f64.  Every point is owned by
// one wave and receives its contributions in canonical order: bitwise the
// oracle's sequential sum over the sorted list.
template <int NDIM, int K>
__global__ __launch_bounds__(SBLOCK) void k_spread(Params p) {
    using T = KT<K>;
    using S = SShape<NDIM, K>;
    constexpr int W = T::W, FAM = T::FAM, LO = T::LO, HI = T::HI;
    constexpr int B = S::B, SB = S::SB, SBV = S::SBV, NPASS = S::NPASS, NBR = S::NBR, CH = S::CH, NQ = S::NQ;
    constexpr int QW = S::QW, KMAX = S::KMAX, CAP = S::CAP, NWD = S::NWD, RWD = S::RWD, LB = S::LB;
    constexpr int QD = NDIM - 1;  // the quartered dim
    __shared__ double acc[SBV];
    __shared__ double rw[CH * RWD];
    __shared__ int rbase[CH];
    __shared__ int rz[CH];
    __shared__ unsigned long long rm[CH * NPASS];
    __shared__ unsigned long long qbits[NQ * NWD];
    __shared__ int cidx[CAP];
    __shared__ int nid[NBR], nst[NBR], nln[NBR], sst[NBR], soff[NBR], npre[NBR + 1], cnt[KMAX * NQ];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    // this lane's stencil point in each pass: acc offset, weight indices, plane
    int loff[NPASS], wi[NPASS][3], lq[NPASS];
#pragma unroll
    for (int ps = 0; ps < NPASS; ++ps) {
        const int q = ps * 64 + lane;
        const int i0 = q % W, i1 = (q / W) % W, i2 = NDIM == 3 ? q / (W * W) : 0;
        loff[ps] = i0 + SB * (i1 + (NDIM == 3 ? SB * i2 : 0));
        wi[ps][0] = i0;
        wi[ps][1] = W + i1;
        wi[ps][2] = 2 * W + i2;
        lq[ps] = NDIM == 3 ? i2 : i1;
    }
    const int nc = p.ncomp;
    const int n = p.nsorted;
    const int nitems = p.bg.nbricks / S::GROUP;
    const int G = gridDim.x;
    for (int round = 0; round < nitems; round += G) {
        const int sb = xcd_item(round, G, blockIdx.x);
        if (sb >= nitems) continue;
        int bc0[3];
        brick_coords<NDIM>(p.bg, sb * S::GROUP, bc0);
        int kb0[3] = {0, 0, 0};
#pragma unroll
        for (int d = 0; d < NDIM; ++d) kb0[d] = p.bg.kmin[d] + bc0[d] * B;

        __syncthreads();  // the previous item is done with the neighbourhood tables
        if (tid < NBR) {
            const int o[3] = {tid & 3, (tid >> 2) & 3, NDIM == 3 ? (tid >> 4) : 1};
            int q[3] = {bc0[0] + o[0] - 1, bc0[1] + o[1] - 1, NDIM == 3 ? bc0[2] + o[2] - 1 : 0};
            bool valid = true;
            for (int d = 0; d < NDIM; ++d) valid = valid && q[d] >= 0 && q[d] < p.bg.nb[d];
            int id = INT_MAX, st = 0, ln = 0;
            if (valid) {
                id = brick_id<NDIM>(p.bg, q);
                st = p.brick_start[id];
                ln = p.brick_start[id + 1] - st;
            }
            nid[tid] = id;
            nst[tid] = st;
            nln[tid] = ln;
        }
        __syncthreads();
        if (tid < NBR) {
            // canonical order = increasing brick id: rank sort of the neighbourhood
            const int my = nid[tid];
            int rank = 0;
            for (int k = 0; k < NBR; ++k) {
                const int o = nid[k];
                rank += (o < my) || (o == my && k < tid);
            }
            sst[rank] = nst[tid];
            soff[rank] = tid;  // packed 2-bit offsets (+1) of the brick
            npre[rank + 1] = nln[tid];
        }
        __syncthreads();
        if (tid == 0) {
            npre[0] = 0;
            for (int k = 0; k < NBR; ++k) npre[k + 1] += npre[k];
        }
        __syncthreads();
        const int total = npre[NBR];
        if (total == 0) continue;
        const int npasses = (total + CAP - 1) / CAP;
        int ncand = 0;

        for (int c = 0; c < nc; ++c) {
            const CompDesc& cd = p.comp[c];
            bool inside = true;
#pragma unroll
            for (int d = 0; d < NDIM; ++d) inside = inside && kb0[d] >= cd.lo[d] && kb0[d] + SB - 1 <= cd.hi[d];
            // u_old of the super-brick's points
            const int64_t o0 = (int64_t)(kb0[0] - cd.lo[0]) + (int64_t)(kb0[1] - cd.lo[1]) * cd.s1 +
                               (NDIM == 3 ? (int64_t)(kb0[2] - cd.lo[2]) * cd.s2 : 0);
            {
                double v[S::NACC];
#pragma unroll
                for (int k = 0; k < S::NACC; ++k) {
                    const int q = tid + k * SBLOCK;
                    const int i0 = q % SB, i1 = (q / SB) % SB, i2 = NDIM == 3 ? q / (SB * SB) : 0;
                    v[k] = 0.0;
                    if (inside) {
                        v[k] = cd.u[o0 + i0 + (int64_t)i1 * cd.s1 + (NDIM == 3 ? (int64_t)i2 * cd.s2 : 0)];
                    } else {
                        const int g0 = kb0[0] + i0, g1 = kb0[1] + i1, g2 = kb0[2] + i2;
                        bool in = g0 >= cd.lo[0] && g0 <= cd.hi[0] && g1 >= cd.lo[1] && g1 <= cd.hi[1];
                        if (NDIM == 3) in = in && g2 >= cd.lo[2] && g2 <= cd.hi[2];
                        if (in)
                            v[k] = cd.u[(int64_t)(g0 - cd.lo[0]) + (int64_t)(g1 - cd.lo[1]) * cd.s1 +
                                        (NDIM == 3 ? (int64_t)(g2 - cd.lo[2]) * cd.s2 : 0)];
                    }
                }
#pragma unroll
                for (int k = 0; k < S::NACC; ++k) acc[tid + k * SBLOCK] = v[k];
            }

            for (int pass = 0; pass < npasses; ++pass) {
                if (npasses > 1 || c == 0) {
                    // ---- filter up to CAP entries: every key load in flight at once
                    __syncthreads();  // cidx / cnt are free
                    unsigned key[KMAX];
                    int eidx[KMAX], ro[KMAX];
#pragma unroll
                    for (int k = 0; k < KMAX; ++k) {
                        const int e = pass * CAP + k * SBLOCK + tid;
                        key[k] = 0u;
                        eidx[k] = -1;
                        ro[k] = 0;
                        if (e < total) {
                            int lo = 0, hi = NBR - 1;  // largest j with npre[j] <= e
                            while (lo < hi) {
                                const int mid = (lo + hi + 1) >> 1;
                                if (npre[mid] <= e) lo = mid;
                                else hi = mid - 1;
                            }
                            eidx[k] = sst[lo] + (e - npre[lo]);
                            ro[k] = soff[lo];
                            key[k] = p.sorted_key[eidx[k]];
                        }
                    }
                    unsigned long long bal[KMAX];
#pragma unroll
                    for (int k = 0; k < KMAX; ++k) {
                        bool cand = eidx[k] >= 0;
                        const unsigned loc = key[k];
#pragma unroll
                        for (int d = 0; d < NDIM; ++d) {
                            // key cell relative to the super-brick's first cell
                            const int rel = (((ro[k] >> (2 * d)) & 3) - 1) * B + (int)((loc >> (LB * d)) & (B - 1));
                            cand = cand && rel >= -HI && rel <= SB - 1 - LO;
                        }
                        bal[k] = __ballot(cand);
                        if (!cand) eidx[k] = -1;
                        if (lane == 0) cnt[k * NQ + wave] = __popcll(bal[k]);
                    }
                    __syncthreads();
                    // ordered compaction: entry order is (k, wave, lane)
                    ncand = 0;
                    for (int k = 0; k < KMAX * NQ; ++k) ncand += cnt[k];
#pragma unroll
                    for (int k = 0; k < KMAX; ++k) {
                        if (eidx[k] >= 0) {
                            int pos = 0;
                            for (int j = 0; j < k * NQ + wave; ++j) pos += cnt[j];
                            pos += __popcll(bal[k] & ((1ull << lane) - 1ull));
                            cidx[pos] = eidx[k];
                        }
                    }
                }

                for (int cb0 = 0; cb0 < ncand; cb0 += CH) {
                    __syncthreads();  // cidx / acc written, previous chunk consumed
                    const int nch = min(CH, ncand - cb0);
                    if (tid < CH) {
                        // ---- prep: this candidate's stencil in component c's frame
                        unsigned qm = 0u;
                        if (tid < nch) {
                            const int idx = cidx[cb0 + tid];
                            double Xs[NDIM];
#pragma unroll
                            for (int d = 0; d < NDIM; ++d) Xs[d] = p.sorted_X[(int64_t)NDIM * idx + d];
                            const double F = p.sorted_F[(int64_t)c * n + idx];
                            const int s = FAM == 2 ? p.sorted_s[idx] : 0;
                            St<W> st[NDIM];
                            marker_stencils_x<NDIM, K>(p, cd, Xs, s, st);
                            double* r = rw + tid * RWD;
                            unsigned vm[3] = {0u, 0u, NDIM == 3 ? 0u : 1u};  // valid stencil indices per dim
                            int cbv = 0, mul = 1;
#pragma unroll
                            for (int d = 0; d < NDIM; ++d) {
                                // binning invariant: the stencil lies in [key + LO, key + HI]
                                const int kc = key_anchor<K>((Xs[d] - p.bg.xlo[d]) / p.bg.dx[d]) + p.bg.ilower[d];
                                if (st[d].ist <= st[d].isp &&
                                    (st[d].icl + st[d].ist < kc + LO || st[d].icl + st[d].isp > kc + HI))
                                    atomicOr(p.err, 2);
#pragma unroll
                                for (int i = 0; i < W; ++i) {
                                    const int lc = st[d].icl + i - kb0[d];
                                    if (i >= st[d].ist && i <= st[d].isp && lc >= 0 && lc < SB) vm[d] |= 1u << i;
                                    // closed form: wz = w2/(dx0*dx1*dx2) (f.m4:1486); 2-D wy = w1/(dx0*dx1)
                                    r[d * W + i] = (FAM == 0 && d == NDIM - 1) ? st[d].w[i] / p.h3 : st[d].w[i];
                                }
                                cbv += (st[d].icl - kb0[d]) * mul;
                                mul *= SB;
                            }
                            r[NDIM * W] = F;
                            rbase[tid] = cbv;
                            const int zrel = st[QD].icl - kb0[QD];
                            rz[tid] = zrel;
                            // lane masks of the valid stencil points, pass by pass
                            unsigned long long m[NPASS];
#pragma unroll
                            for (int ps = 0; ps < NPASS; ++ps) m[ps] = 0ull;
                            const int n2 = NDIM == 3 ? W : 1;
                            for (int i2 = 0; i2 < n2; ++i2) {
                                if (!((vm[2] >> i2) & 1u)) continue;
                                for (int i1 = 0; i1 < W; ++i1) {
                                    if (!((vm[1] >> i1) & 1u)) continue;
                                    const int q0 = W * i1 + W * W * i2;
                                    const unsigned long long row = (unsigned long long)vm[0];
#pragma unroll
                                    for (int ps = 0; ps < NPASS; ++ps) {
                                        const int sh = q0 - 64 * ps;
                                        if (sh >= 0 && sh < 64) m[ps] |= row << sh;
                                        else if (sh < 0 && sh > -W) m[ps] |= row >> (-sh);
                                    }
                                }
                            }
                            unsigned long long any = 0ull;
#pragma unroll
                            for (int ps = 0; ps < NPASS; ++ps) {
                                rm[tid * NPASS + ps] = m[ps];
                                any |= m[ps];
                            }
                            if (any) {
#pragma unroll
                                for (int i = 0; i < W; ++i)
                                    if ((vm[QD] >> i) & 1u) qm |= 1u << ((zrel + i) / QW);
                            }
                        }
#pragma unroll
                        for (int q = 0; q < NQ; ++q) {
                            const unsigned long long b = __ballot((qm >> q) & 1u);
                            if (lane == 0) qbits[q * NWD + wave] = b;
                        }
                    }
                    __syncthreads();
                    // ---- wave `wave` adds, in canonical order, the points of its
                    // quarter [qlo, qlo + QW) of the candidates whose bit is set
                    const int qlo = wave * QW;
                    for (int wd = 0; wd < NWD; ++wd) {
                        unsigned long long bits = qbits[wave * NWD + wd];
                        bits = ((unsigned long long)__builtin_amdgcn_readfirstlane((unsigned)(bits >> 32)) << 32) |
                               (unsigned)__builtin_amdgcn_readfirstlane((unsigned)bits);
                        while (bits) {
                            // two candidates per trip: both records are read before either add
                            const int ca = wd * 64 + __builtin_ctzll(bits);
                            bits &= bits - 1ull;
                            const bool two = bits != 0ull;
                            const int cb = two ? wd * 64 + __builtin_ctzll(bits) : ca;
                            if (two) bits &= bits - 1ull;
                            double contrib[2][NPASS];
                            bool on[2][NPASS];
                            int addr[2][NPASS];
#pragma unroll
                            for (int h = 0; h < 2; ++h) {
                                const int ci = h ? cb : ca;
                                const double* r = rw + ci * RWD;
                                const double F = r[NDIM * W];
                                const int base = rbase[ci], zrel = rz[ci];
#pragma unroll
                                for (int ps = 0; ps < NPASS; ++ps) {
                                    const unsigned long long m = rm[ci * NPASS + ps];
                                    on[h][ps] = ((m >> lane) & 1ull) && (unsigned)(zrel + lq[ps] - qlo) < (unsigned)QW;
                                    addr[h][ps] = base + loff[ps];
                                    double cv;
                                    if constexpr (FAM == 3) {
                                        cv = F / p.h3;  // f.m4:170-171
                                    } else if constexpr (FAM == 0) {
                                        double wt;
                                        if constexpr (NDIM == 3)
                                            wt = r[wi[ps][0]] * (r[wi[ps][1]] * r[wi[ps][2]]);  // f.m4:1485-1492
                                        else
                                            wt = r[wi[ps][0]] * r[wi[ps][1]];
                                        cv = wt * F;  // f.m4:1512-1513
                                    } else {
                                        if constexpr (NDIM == 3)
                                            cv = r[wi[ps][0]] * r[wi[ps][1]] * r[wi[ps][2]] * F / p.h3;
                                        else
                                            cv = r[wi[ps][0]] * r[wi[ps][1]] * F / p.h3;  // f.m4:668-672
                                    }
                                    contrib[h][ps] = cv;
                                }
                            }
#pragma unroll
                            for (int h = 0; h < 2; ++h) {
                                if (h == 1 && !two) break;
#pragma unroll
                                for (int ps = 0; ps < NPASS; ++ps)
                                    if (on[h][ps])
                                        __hip_atomic_fetch_add(&acc[addr[h][ps]], contrib[h][ps], __ATOMIC_RELAXED,
                                                               __HIP_MEMORY_SCOPE_WORKGROUP);
                            }
                        }
                    }
                }
            }
            __syncthreads();
            // write back the super-brick's points
#pragma unroll
            for (int k = 0; k < S::NACC; ++k) {
                const int q = tid + k * SBLOCK;
                const int i0 = q % SB, i1 = (q / SB) % SB, i2 = NDIM == 3 ? q / (SB * SB) : 0;
                if (inside) {
                    cd.u[o0 + i0 + (int64_t)i1 * cd.s1 + (NDIM == 3 ? (int64_t)i2 * cd.s2 : 0)] = acc[q];
                } else {
                    const int g0 = kb0[0] + i0, g1 = kb0[1] + i1, g2 = kb0[2] + i2;
                    bool in = g0 >= cd.lo[0] && g0 <= cd.hi[0] && g1 >= cd.lo[1] && g1 <= cd.hi[1];
                    if (NDIM == 3) in = in && g2 >= cd.lo[2] && g2 <= cd.hi[2];
                    if (in)
                        cd.u[(int64_t)(g0 - cd.lo[0]) + (int64_t)(g1 - cd.lo[1]) * cd.s1 +
                             (NDIM == 3 ? (int64_t)(g2 - cd.lo[2]) * cd.s2 : 0)] = acc[q];
                }
            }
        }
    }
}

template <int NDIM, int K>
hipError_t launch_spread_t(const Params& p, hipStream_t s, hipEvent_t ev0, hipEvent_t ev1) {
    using S = SShape<NDIM, K>;
    if (ev0) (void)hipEventRecord(ev0, s);
    if (p.nsorted > 0)
        hipLaunchKernelGGL(k_gather_F, dim3((p.nsorted + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, s, p, p.nsorted,
                           const_cast<double*>(p.sorted_F));
    const long items = (long)(p.bg.nbricks / S::GROUP);
    hipLaunchKernelGGL((k_spread<NDIM, K>), dim3(grid_for(items, 64)), dim3(SBLOCK), 0, s, p);
    if (ev1) (void)hipEventRecord(ev1, s);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// dispatch
// ---------------------------------------------------------------------------
#define IBTK_LE_DISPATCH(NDIMV, KV, CALL)                                     \
    switch (KV) {                                                             \
    case K_PIECEWISE_CONSTANT: return CALL<NDIMV, K_PIECEWISE_CONSTANT>;      \
    case K_DISCONTINUOUS_LINEAR: return CALL<NDIMV, K_DISCONTINUOUS_LINEAR>;  \
    case K_PIECEWISE_LINEAR: return CALL<NDIMV, K_PIECEWISE_LINEAR>;          \
    case K_PIECEWISE_CUBIC: return CALL<NDIMV, K_PIECEWISE_CUBIC>;            \
    case K_IB_3: return CALL<NDIMV, K_IB_3>;                                  \
    case K_IB_4: return CALL<NDIMV, K_IB_4>;                                  \
    case K_IB_4_W8: return CALL<NDIMV, K_IB_4_W8>;                            \
    case K_IB_6: return CALL<NDIMV, K_IB_6>;                                  \
    case K_BSPLINE_4: return CALL<NDIMV, K_BSPLINE_4>;                        \
    default: return nullptr;                                                  \
    }

using BinFn = hipError_t (*)(const Params&, int, unsigned*, int*, hipStream_t);
using InterpFn = hipError_t (*)(const Params&, int, hipStream_t, hipEvent_t, hipEvent_t);
using SpreadFn = hipError_t (*)(const Params&, hipStream_t, hipEvent_t, hipEvent_t);

template <int NDIM> static BinFn pick_bin(int k) { IBTK_LE_DISPATCH(NDIM, k, launch_bin_t) }
template <int NDIM> static InterpFn pick_interp(int k) { IBTK_LE_DISPATCH(NDIM, k, launch_interp_t) }
template <int NDIM> static SpreadFn pick_spread(int k) { IBTK_LE_DISPATCH(NDIM, k, launch_spread_t) }

hipError_t launch_bin(int ndim, int kernel, const Params& p, int n, unsigned* keys, int* vals, hipStream_t s) {
    BinFn f = ndim == 3 ? pick_bin<3>(kernel) : pick_bin<2>(kernel);
    return f ? f(p, n, keys, vals, s) : hipErrorInvalidValue;
}
hipError_t launch_brick_start(const unsigned* keys, int n, int nbricks, int shift, int* bs, hipStream_t s) {
    hipLaunchKernelGGL(k_brick_start, dim3((n + 1 + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, s, keys, n, nbricks, shift,
                       bs);
    return hipGetLastError();
}
hipError_t launch_gather_sorted(int ndim, const Params& p, int n, int* sorted_s, double* sorted_X, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    if (ndim == 3)
        hipLaunchKernelGGL(k_gather_sorted<3>, dim3((n + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, s, p, n, sorted_s,
                           sorted_X);
    else
        hipLaunchKernelGGL(k_gather_sorted<2>, dim3((n + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, s, p, n, sorted_s,
                           sorted_X);
    return hipGetLastError();
}
hipError_t launch_interp(int ndim, int kernel, const Params& p, int n, hipStream_t s, hipEvent_t ev0,
                         hipEvent_t ev1) {
    InterpFn f = ndim == 3 ? pick_interp<3>(kernel) : pick_interp<2>(kernel);
    return f ? f(p, n, s, ev0, ev1) : hipErrorInvalidValue;
}
hipError_t launch_spread(int ndim, int kernel, const Params& p, hipStream_t s, hipEvent_t ev0, hipEvent_t ev1) {
    SpreadFn f = ndim == 3 ? pick_spread<3>(kernel) : pick_spread<2>(kernel);
    return f ? f(p, s, ev0, ev1) : hipErrorInvalidValue;
}

}  // namespace ibtk_le
