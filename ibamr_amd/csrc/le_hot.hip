// le_hot.hip -- the 2-D hot path on CDNA4 (gfx950): brick binning,
// interpolation and spreading.  Replaces the l-loops of
// ibtk/src/lagrangian/fortran/lagrangian_interaction2d.f.m4.  (The 3-D path is
// le_sweep.hip's column sweeps; the templates below are written for NDIM = 2
// or 3 but only NDIM = 2 is instantiated -- see the dispatchers at the end.)
//
// Work decomposition:
//  * bin: key = brick id (tiled, le_bricks.h) << 8 | cell-in-brick of the
//    marker's cell-frame stencil anchor (16^2-cell bricks); stable device radix
//    sort; brick CSR; then one coalescing pass writes the sorted marker index
//    and the sorted shifted position X(s)+Xshift(l), so the interp/spread
//    kernels read their markers contiguously.
//  * interp: one workgroup item = (brick, component).  The union stencil region
//    of the brick's markers is loaded from HBM with every load of a thread in
//    flight at once and staged in LDS; one thread per marker then sums its W^2
//    stencil from LDS in the Fortran loop order, so the result is bitwise the
//    oracle's.
//  * spread: one workgroup item = (super-brick of 2x2 bricks, component).  The
//    workgroup loads u_old of its points into LDS, walks the sorted entries of
//    the surrounding bricks in canonical (sorted) order, keeps those whose
//    stencil can reach the super-brick (parallel filter + ordered block
//    compaction), computes their 1-D weights in parallel, and one wave then adds
//    candidate after candidate with lane = stencil point (ds_add_f64 into LDS).
//    Each grid point therefore receives its contributions in list order exactly
//    like the Fortran's sequential l-loop: no global atomics, deterministic,
//    bitwise the oracle's on the same list.
#include <hip/hip_runtime.h>

#include <climits>
#include <cstdio>
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

// bs[b] = first sorted position whose bucket (key >> shift) >= b, for b in [0, nbuckets]
// (buckets = cell planes of bricks: plane_start).
__global__ __launch_bounds__(BLOCK) void k_brick_start(const unsigned* keys, int n, int nbricks, int shift, int* bs) {  // nbricks = nbuckets
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
// Interpolation work item: a group of GB consecutive bricks (2x2[x1] bricks, or
// one brick for the wide kernels) and all its markers; per component the union
// stencil region of the group, R0 x R1 [x R2] points, is staged in LDS.
template <int NDIM, int K> struct IShape {
    using T = KT<K>;
    static constexpr int B = BrickT<NDIM>::B;
    static constexpr int GB = T::W <= 4 ? 4 : 1;   // bricks per item (ids b..b+GB-1: 2x2[x1] in Morton order)
    static constexpr int E0 = GB == 4 ? 2 * B : B;  // anchor extent of the item in dims 0 and 1
    static constexpr int R0 = E0 + T::HI - T::LO, R1 = R0;
    static constexpr int R2 = NDIM == 3 ? B + T::HI - T::LO : 1;
    static constexpr int RV = R0 * R1 * R2;
    static constexpr int NL = (RV + BLOCK - 1) / BLOCK;  // staged values per thread
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

// region value loads of component cd for the item whose region starts at r0
template <int NDIM, int K>
__device__ __forceinline__ void stage_load(const CompDesc& cd, const int* r0, double* v) {
    using S = IShape<NDIM, K>;
    constexpr int R0 = S::R0, R1 = S::R1, R2 = S::R2, RV = S::RV;
    bool inside = true;
#pragma unroll
    for (int d = 0; d < NDIM; ++d) {
        const int R = d == 0 ? R0 : (d == 1 ? R1 : R2);
        inside = inside && r0[d] >= cd.lo[d] && r0[d] + R - 1 <= cd.hi[d];
    }
    const int64_t o0 = (int64_t)(r0[0] - cd.lo[0]) + (int64_t)(r0[1] - cd.lo[1]) * cd.s1 +
                       (NDIM == 3 ? (int64_t)(r0[2] - cd.lo[2]) * cd.s2 : 0);
    // (recomputed per item on purpose: hoisted out of the item loop, the 3*NL
    // index registers would stay live through the stencil sums)
    int t = threadIdx.x;
    asm volatile("" : "+v"(t));
#pragma unroll
    for (int k = 0; k < S::NL; ++k) {
        const int q = t + k * BLOCK;
        v[k] = 0.0;
        if (q < RV) {
            const int i0 = q % R0, i1 = (q / R0) % R1, i2 = NDIM == 3 ? q / (R0 * R1) : 0;
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
}

// One workgroup item = GB bricks, every component: the component's region is
// staged in LDS (the next component's loads are in flight while this one is
// summed), then one thread per marker sums its W^NDIM stencil from LDS in the
// Fortran loop order -- bitwise the oracle's value.
template <int NDIM, int K>
__global__ __launch_bounds__(BLOCK) void k_interp(Params p) {
    using T = KT<K>;
    using S = IShape<NDIM, K>;
    constexpr int W = T::W, FAM = T::FAM, B = S::B, R0 = S::R0, R1 = S::R1, R2 = S::R2, NL = S::NL;
    __shared__ double reg[S::RV];
    const int nc = p.ncomp;
    const int nitems = p.bg.nbricks / S::GB;
    const int G = gridDim.x;
    const int tid = threadIdx.x;
    for (int round = 0; round < nitems; round += G) {
        const int it = xcd_item(round, G, blockIdx.x);
        if (it >= nitems) continue;
        const int b0 = it * S::GB;
        const int beg = p.plane_start[b0 * B], end = p.plane_start[(b0 + S::GB) * B];
        if (beg == end) continue;
        int bc[3];
        brick_coords<NDIM>(p.bg, b0, bc);
        int r0[3] = {0, 0, 0};
#pragma unroll
        for (int d = 0; d < NDIM; ++d) r0[d] = p.bg.kmin[d] + bc[d] * B + T::LO;
        // this thread's first marker, kept across the components
        const int e0 = beg + tid;
        int s0 = 0;
        double x0[NDIM];
        if (e0 < end) {
            s0 = p.sorted_s[e0];
#pragma unroll
            for (int d = 0; d < NDIM; ++d) x0[d] = p.sorted_X[(int64_t)NDIM * e0 + d];
        }
        for (int c = 0; c < nc; ++c) {
            const CompDesc& cd = p.comp[c];
            {
                double v[NL];
                stage_load<NDIM, K>(cd, r0, v);
                __syncthreads();  // the previous readers of reg are done
#pragma unroll
                for (int k = 0; k < NL; ++k) {
                    const int q = tid + k * BLOCK;
                    if (q < S::RV) reg[q] = v[k];
                }
                __syncthreads();
            }

            for (int e = e0; e < end; e += BLOCK) {
                int s = s0;
                double xs[NDIM];
#pragma unroll
                for (int d = 0; d < NDIM; ++d) xs[d] = x0[d];
                if (e != e0) {
                    s = p.sorted_s[e];
#pragma unroll
                    for (int d = 0; d < NDIM; ++d) xs[d] = p.sorted_X[(int64_t)NDIM * e + d];
                }
                St<W> st[NDIM];
                marker_stencils_x<NDIM, K>(p, cd, xs, s, st);
                bool ok = true;
#pragma unroll
                for (int d = 0; d < NDIM; ++d) {
                    const int R = d == 0 ? R0 : (d == 1 ? R1 : R2);
                    if (st[d].ist <= st[d].isp)
                        ok = ok && (st[d].icl + st[d].ist >= r0[d]) && (st[d].icl + st[d].isp < r0[d] + R);
                }
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
                        int li = st[0].icl - r0[0] + R0 * (st[1].icl - r0[1]);
                        if (NDIM == 3) li += R0 * R1 * (st[2 % NDIM].icl - r0[2]);
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
                        const int R = d == 0 ? R0 : (d == 1 ? R1 : R2);
                        const int stride = d == 0 ? 1 : (d == 1 ? R0 : R0 * R1);
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
                const int sq = p.qdst ? p.qdst[e] : s;
                if (sq >= 0) p.Qout[(int64_t)p.Q_depth * sq + cd.qcomp] = acc;
            }
        }
    }
}

// Entries binned "outside" (no stencil point can reach any array): V = 0.
__global__ __launch_bounds__(BLOCK) void k_interp_outside(Params p, int n) {
    const int first = p.plane_start[p.bg.nbricks * (p.bg.ndim == 3 ? BRICK3 : BRICK2)];
    for (int e = first + blockIdx.x * BLOCK + threadIdx.x; e < n; e += gridDim.x * BLOCK) {
        const int s = p.qdst ? p.qdst[e] : p.sorted_s[e];
        if (s < 0) continue;
        for (int c = 0; c < p.ncomp; ++c) p.Qout[(int64_t)p.Q_depth * s + p.comp[c].qcomp] = 0.0;
    }
}

template <int NDIM, int K>
hipError_t launch_interp_t(const Params& p, int n, hipStream_t s, hipEvent_t ev0, hipEvent_t ev1) {
    using S = IShape<NDIM, K>;
    if (ev0) (void)hipEventRecord(ev0, s);
    const long items = (long)(p.bg.nbricks / S::GB);
    hipLaunchKernelGGL((k_interp<NDIM, K>), dim3(grid_for(items, 64)), dim3(BLOCK), 0, s, p);
    if (ev1) (void)hipEventRecord(ev1, s);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    if (n > 0) hipLaunchKernelGGL(k_interp_outside, dim3(64), dim3(BLOCK), 0, s, p, n);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// spreading
// ---------------------------------------------------------------------------
// Work item: one super-brick (2^NDIM bricks: 16^3 cells in 3-D, 32^2 in 2-D).
// Its candidates -- the markers whose stencil can reach it -- are grouped into
// "classes" of CW anchor planes along the last dim.  A class's stencils lie in
// CW + HI - LO consecutive planes, so classes NPH apart never touch the same
// grid point: in phase ph the waves of the workgroup take the classes
// ph, ph + NPH, ... concurrently, phases separated by a barrier.
template <int NDIM, int K> struct SShape {
    using BT = BrickT<NDIM>;
    static constexpr int B = BT::B, SB = BT::SB, SBV = BT::SBV, GROUP = BT::GROUP;
    static constexpr int W = KT<K>::W, LO = KT<K>::LO, HI = KT<K>::HI;
    static constexpr int NQ = SBLOCK / 64;                                // waves
    static constexpr int NBR = NDIM == 3 ? 64 : 16;                       // neighbourhood bricks (4 per dim)
    static constexpr int KMAX = 4;                                        // entries per thread per list sub-pass
    static constexpr int CW = 2;                                          // anchor planes per class
    static constexpr int NCLS = (SB - 1 + HI - LO) / CW + 1;              // classes of a super-brick
    static constexpr int NPH = 1 + (HI - LO + CW - 1) / CW;               // phases
    static constexpr int NACC = SBV / SBLOCK;                             // u values per thread
    static constexpr int LB = NDIM == 3 ? 3 : 4;                          // log2(B)
    static constexpr int MAXOFF = NDIM == 3 ? (W - 1) * (1 + SB + SB * SB) : (W - 1) * (1 + SB);
    static constexpr int TRASH = 64 + MAXOFF + 1;                         // per-lane sink of masked points
    static_assert(HI <= B && -LO <= B, "a stencil must not reach beyond the neighbouring brick");
    static_assert(NPH * CW >= CW + HI - LO, "classes of one phase must be disjoint");
};

// The sorted entries that can reach super-brick `sb`: for each of the 4^NDIM
// bricks around it, the run of its cell planes (along the last dim; entries of a
// brick are sorted by cell, last dim slowest) whose anchors can reach the
// super-brick, the runs ranked by brick id (= canonical order).  Returns the
// number of entries; npre[] are the runs' prefix offsets, sst[] their starts,
// soff[] the packed 2-bit (offset + 1) of their bricks.
template <int NDIM, int K>
__device__ int neighbourhood(const Params& p, int sb, int* nid, int* nst, int* nln, int* sst, int* soff, int* npre) {
    using S = SShape<NDIM, K>;
    constexpr int B = S::B, NBR = S::NBR, HI = S::HI, LO = S::LO;
    const int tid = threadIdx.x;
    int bc0[3];
    brick_coords<NDIM>(p.bg, sb * S::GROUP, bc0);
    __syncthreads();  // the tables are free
    if (tid < NBR) {
        const int o[3] = {tid & 3, (tid >> 2) & 3, NDIM == 3 ? (tid >> 4) : 0};
        int q[3] = {bc0[0] + o[0] - 1, bc0[1] + o[1] - 1, NDIM == 3 ? bc0[2] + o[2] - 1 : 0};
        bool valid = true;
        for (int d = 0; d < NDIM; ++d) valid = valid && q[d] >= 0 && q[d] < p.bg.nb[d];
        const int ol = o[NDIM - 1];
        const int plo = ol == 0 ? B - HI : 0;       // planes whose anchors reach the super-brick
        const int phi = ol == 3 ? -LO - 1 : B - 1;  // (inclusive)
        int id = INT_MAX, st = 0, ln = 0;
        if (valid) {
            id = brick_id<NDIM>(p.bg, q);
            st = p.plane_start[id * B + plo];
            ln = p.plane_start[id * B + phi + 1] - st;
        }
        nid[tid] = id;
        nst[tid] = st;
        nln[tid] = ln;
    }
    __syncthreads();
    if (tid < NBR) {
        const int my = nid[tid];
        int rank = 0;
        for (int k = 0; k < NBR; ++k) {
            const int o = nid[k];
            rank += (o < my) || (o == my && k < tid);
        }
        sst[rank] = nst[tid];
        soff[rank] = tid;
        npre[rank + 1] = nln[tid];
    }
    __syncthreads();
    if (tid == 0) {
        npre[0] = 0;
        for (int k = 0; k < NBR; ++k) npre[k + 1] += npre[k];
    }
    __syncthreads();
    return npre[NBR];
}

// entry e of the neighbourhood -> sorted index (and the packed brick offset)
template <int NBR> __device__ __forceinline__ int entry_of(int e, const int* npre, const int* sst, const int* soff, int& ro) {
    int lo = 0, hi = NBR - 1;  // largest j with npre[j] <= e
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (npre[mid] <= e) lo = mid;
        else hi = mid - 1;
    }
    ro = soff[lo];
    return sst[lo] + (e - npre[lo]);
}

// class of the entry with this key (in the brick at packed offset ro) for the
// super-brick, or -1 if its stencil cannot reach the super-brick
template <int NDIM, int K> __device__ __forceinline__ int cand_class(unsigned key, int ro) {
    using S = SShape<NDIM, K>;
    bool cand = true;
    int rl = 0;
#pragma unroll
    for (int d = 0; d < NDIM; ++d) {
        const int rel = (((ro >> (2 * d)) & 3) - 1) * S::B + (int)((key >> (S::LB * d)) & (S::B - 1));
        cand = cand && rel >= -S::HI && rel <= S::SB - 1 - S::LO;
        rl = rel;
    }
    return cand ? (rl + S::HI) / S::CW : -1;
}

// Candidate lists, built once per binning: for super-brick sb and class k, the
// entries of that class whose stencil can reach sb, in canonical order, at
// [off[sb*NCLS + k], off[sb*NCLS + k + 1]).  Pass 1 counts, an exclusive scan
// gives the offsets, pass 2 writes (ordered block compaction per class).
template <int NDIM, int K, bool WRITE>
__global__ __launch_bounds__(SBLOCK) void k_cand(Params p, int* counts_or_offs, int* out) {
    using S = SShape<NDIM, K>;
    constexpr int NBR = S::NBR, KMAX = S::KMAX, NQ = S::NQ, NCLS = S::NCLS;
    __shared__ int nid[NBR], nst[NBR], nln[NBR], sst[NBR], soff[NBR], npre[NBR + 1];
    __shared__ int cnt[KMAX * NQ * NCLS];
    __shared__ int cbase[NCLS];
    const int nitems = p.bg.nbricks / S::GROUP;
    const int sb = xcd_item(0, gridDim.x, blockIdx.x);
    if (sb >= nitems) return;
    const int total = neighbourhood<NDIM, K>(p, sb, nid, nst, nln, sst, soff, npre);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (!WRITE) {
        if (tid < NCLS) cbase[tid] = 0;
        __syncthreads();
        for (int e = tid; e < total; e += SBLOCK) {
            int ro;
            const int idx = entry_of<NBR>(e, npre, sst, soff, ro);
            const int k = cand_class<NDIM, K>(p.sorted_key[idx], ro);
            if (k >= 0) atomicAdd(&cbase[k], 1);
        }
        __syncthreads();
        if (tid < NCLS) counts_or_offs[sb * NCLS + tid] = cbase[tid];
        return;
    }
    if (tid < NCLS) cbase[tid] = counts_or_offs[sb * NCLS + tid];
    for (int e0 = 0; e0 < total; e0 += KMAX * SBLOCK) {
        int eidx[KMAX], cls[KMAX];
#pragma unroll
        for (int k = 0; k < KMAX; ++k) {
            const int e = e0 + k * SBLOCK + tid;
            eidx[k] = -1;
            cls[k] = -1;
            int ro = 0;
            if (e < total) eidx[k] = entry_of<NBR>(e, npre, sst, soff, ro);
            if (eidx[k] >= 0) cls[k] = cand_class<NDIM, K>(p.sorted_key[eidx[k]], ro);
        }
        // per (sub-pass slot, wave, class) counts; entry order is (k, wave, lane)
        unsigned long long mine[KMAX];
#pragma unroll
        for (int k = 0; k < KMAX; ++k) {
            mine[k] = 0ull;
            for (int c = 0; c < NCLS; ++c) {
                const unsigned long long b = __ballot(cls[k] == c);
                if (cls[k] == c) mine[k] = b;
                if (lane == 0) cnt[(k * NQ + wave) * NCLS + c] = __popcll(b);
            }
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < KMAX; ++k) {
            const int c = cls[k];
            if (c >= 0) {
                int pos = cbase[c];
                for (int j = 0; j < k * NQ + wave; ++j) pos += cnt[j * NCLS + c];
                pos += __popcll(mine[k] & ((1ull << lane) - 1ull));
                out[pos] = eidx[k];
            }
        }
        __syncthreads();
        if (tid < NCLS) {
            int t = 0;
            for (int j = 0; j < KMAX * NQ; ++j) t += cnt[j * NCLS + tid];
            cbase[tid] += t;
        }
        __syncthreads();
    }
}

// sorted_F[c * n + e] = Q(qcomp_c, s(e)): the spread values in sorted order, so
// the spread kernel's loads of them are contiguous and not behind the s load.
__global__ __launch_bounds__(BLOCK) void k_gather_F(Params p, int n, double* out) {
    const int e = blockIdx.x * BLOCK + threadIdx.x;
    if (e >= n) return;
    const int s = p.sorted_s[e];
    // density-weighted spread: F ds rounded once, as LDataManager.cpp:446-451 forms it
    const double w = p.ds ? p.ds[s] : 1.0;
    for (int c = 0; c < p.ncomp; ++c) {
        const double v = p.Qin[(int64_t)p.Q_depth * s + p.comp[c].qcomp];
        out[(int64_t)c * n + e] = p.ds ? v * w : v;
    }
}

// Spread of one super-brick, component after component: u_old goes to LDS; in
// each phase every wave takes its classes' candidates 64 at a time, one per
// lane: the lane computes the candidate's 1-D weights in registers and adds its
// W^NDIM stencil points to LDS (ds_add_f64, one instruction per stencil point
// for the 64 candidates; points outside the super-brick or clipped by the
// ghost box go to a per-lane sink).  A grid point receives its contributions
// in a fixed order -- phase, class list order, stencil point, lane -- so the
// result is deterministic run to run (and equal to the sequential Fortran sum
// up to reassociation).
template <int NDIM, int K>
__global__ __launch_bounds__(SBLOCK) void k_spread(Params p) {
    using T = KT<K>;
    using S = SShape<NDIM, K>;
    constexpr int W = T::W, FAM = T::FAM, LO = T::LO, HI = T::HI;
    constexpr int B = S::B, SB = S::SB, SBV = S::SBV, NQ = S::NQ, NCLS = S::NCLS, NPH = S::NPH, CW = S::CW;
    constexpr int QD = NDIM - 1;
    __shared__ double acc[SBV + S::TRASH];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int nc = p.ncomp;
    const int n = p.nsorted;
    const int nitems = p.bg.nbricks / S::GROUP;
    const int G = gridDim.x;
    const int sink = SBV + lane;  // this lane's sink slot
    for (int round = 0; round < nitems; round += G) {
        const int sb = xcd_item(round, G, blockIdx.x);
        if (sb >= nitems) continue;
        const int* off = p.cand_off + (int64_t)sb * NCLS;
        if (off[NCLS] == off[0]) continue;  // no candidates: u unchanged
        int bc0[3];
        brick_coords<NDIM>(p.bg, sb * S::GROUP, bc0);
        int kb0[3] = {0, 0, 0};
#pragma unroll
        for (int d = 0; d < NDIM; ++d) kb0[d] = p.bg.kmin[d] + bc0[d] * B;

        // the first 64 candidates of this wave's first class in each phase:
        // indices and positions loaded once, kept across the components
        int idx0[NPH];
        double X0[NPH][NDIM];
#pragma unroll
        for (int ph = 0; ph < NPH; ++ph) {
            const int k = ph + NPH * wave;
            idx0[ph] = -1;
            if (k < NCLS) {
                const int e = off[k] + lane;
                if (e < off[k + 1]) idx0[ph] = p.cand_idx[e];
            }
        }
#pragma unroll
        for (int ph = 0; ph < NPH; ++ph)
#pragma unroll
            for (int d = 0; d < NDIM; ++d) X0[ph][d] = idx0[ph] >= 0 ? p.sorted_X[(int64_t)NDIM * idx0[ph] + d] : 0.0;

        for (int c = 0; c < nc; ++c) {
            const CompDesc& cd = p.comp[c];
            bool inside = true;
#pragma unroll
            for (int d = 0; d < NDIM; ++d) inside = inside && kb0[d] >= cd.lo[d] && kb0[d] + SB - 1 <= cd.hi[d];
            const int64_t o0 = (int64_t)(kb0[0] - cd.lo[0]) + (int64_t)(kb0[1] - cd.lo[1]) * cd.s1 +
                               (NDIM == 3 ? (int64_t)(kb0[2] - cd.lo[2]) * cd.s2 : 0);
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
            double F0[NPH];
#pragma unroll
            for (int ph = 0; ph < NPH; ++ph) F0[ph] = idx0[ph] >= 0 ? p.sorted_F[(int64_t)c * n + idx0[ph]] : 0.0;
            __syncthreads();  // the previous component's write-back has read acc
#pragma unroll
            for (int k = 0; k < S::NACC; ++k) acc[tid + k * SBLOCK] = v[k];
            __syncthreads();

#pragma unroll
            for (int ph = 0; ph < NPH; ++ph) {
                for (int k = ph + NPH * wave; k < NCLS; k += NPH * NQ) {
                    const int first = k == ph + NPH * wave;
                    for (int e0 = off[k]; e0 < off[k + 1]; e0 += 64) {
                        // ---- this lane's candidate
                        int idx;
                        double Xs[NDIM], F;
                        if (first && e0 == off[k]) {
                            idx = idx0[ph];
#pragma unroll
                            for (int d = 0; d < NDIM; ++d) Xs[d] = X0[ph][d];
                            F = F0[ph];
                        } else {
                            const int e = e0 + lane;
                            idx = e < off[k + 1] ? p.cand_idx[e] : -1;
#pragma unroll
                            for (int d = 0; d < NDIM; ++d) Xs[d] = idx >= 0 ? p.sorted_X[(int64_t)NDIM * idx + d] : 0.0;
                            F = idx >= 0 ? p.sorted_F[(int64_t)c * n + idx] : 0.0;
                        }
                        const int s = (FAM == 2 && idx >= 0) ? p.sorted_s[idx] : 0;
                        St<W> st[NDIM];
                        marker_stencils_x<NDIM, K>(p, cd, Xs, s, st);
                        // valid stencil indices per dim: inside the clip range and the super-brick
                        unsigned vm[3] = {0u, 0u, NDIM == 3 ? 0u : 1u};
                        double w[NDIM][W];
                        int base = 0, mul = 1;
#pragma unroll
                        for (int d = 0; d < NDIM; ++d) {
#pragma unroll
                            for (int i = 0; i < W; ++i) {
                                const int lc = st[d].icl + i - kb0[d];
                                if (idx >= 0 && i >= st[d].ist && i <= st[d].isp && lc >= 0 && lc < SB) vm[d] |= 1u << i;
                                // closed form: wz = w2/(dx0*dx1*dx2) (f.m4:1486); 2-D wy = w1/(dx0*dx1)
                                w[d][i] = (FAM == 0 && d == NDIM - 1) ? st[d].w[i] / p.h3 : st[d].w[i];
                            }
                            base += (st[d].icl - kb0[d]) * mul;
                            mul *= SB;
                        }
                        // class invariant: the stencil's planes lie in the class footprint
                        if (idx >= 0 && st[QD].ist <= st[QD].isp) {
                            const int z0 = st[QD].icl + st[QD].ist - kb0[QD], z1 = st[QD].icl + st[QD].isp - kb0[QD];
                            if (z0 < k * CW - HI + LO || z1 > k * CW + CW - 1) atomicOr(p.err, 2);
                        }
                        // ---- add the W^NDIM points (lane = candidate)
                        if constexpr (NDIM == 3) {
#pragma unroll
                            for (int i2 = 0; i2 < W; ++i2) {
#pragma unroll
                                for (int i1 = 0; i1 < W; ++i1) {
                                    const bool v12 = ((vm[1] >> i1) & (vm[2] >> i2) & 1u) != 0u;
                                    double w12 = 0.0;
                                    if constexpr (FAM == 0) w12 = w[1][i1] * w[2][i2];  // f.m4:1485-1492
#pragma unroll
                                    for (int i0 = 0; i0 < W; ++i0) {
                                        const bool on = v12 && ((vm[0] >> i0) & 1u);
                                        double cv;
                                        if constexpr (FAM == 3) cv = F / p.h3;  // f.m4:170-171
                                        else if constexpr (FAM == 0) cv = (w[0][i0] * w12) * F;  // f.m4:1512-1513
                                        else cv = w[0][i0] * w[1][i1] * w[2][i2] * F / p.h3;
                                        const int a = on ? base : sink;
                                        __hip_atomic_fetch_add(&acc[a + i0 + SB * (i1 + SB * i2)], cv, __ATOMIC_RELAXED,
                                                               __HIP_MEMORY_SCOPE_WORKGROUP);
                                    }
                                }
                            }
                        } else {
#pragma unroll
                            for (int i1 = 0; i1 < W; ++i1) {
                                const bool v1 = ((vm[1] >> i1) & 1u) != 0u;
#pragma unroll
                                for (int i0 = 0; i0 < W; ++i0) {
                                    const bool on = v1 && ((vm[0] >> i0) & 1u);
                                    double cv;
                                    if constexpr (FAM == 3) cv = F / p.h3;
                                    else if constexpr (FAM == 0) cv = (w[0][i0] * w[1][i1]) * F;
                                    else cv = w[0][i0] * w[1][i1] * F / p.h3;  // f.m4:668-672
                                    const int a = on ? base : sink;
                                    __hip_atomic_fetch_add(&acc[a + i0 + SB * i1], cv, __ATOMIC_RELAXED,
                                                           __HIP_MEMORY_SCOPE_WORKGROUP);
                                }
                            }
                        }
                    }
                }
                __syncthreads();  // phase boundary
            }
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
hipError_t launch_cand_t(const Params& p, bool write, int* counts_or_offs, int* out, hipStream_t s) {
    using S = SShape<NDIM, K>;
    const int items = p.bg.nbricks / S::GROUP;
    if (write)
        hipLaunchKernelGGL((k_cand<NDIM, K, true>), dim3(items), dim3(SBLOCK), 0, s, p, counts_or_offs, out);
    else
        hipLaunchKernelGGL((k_cand<NDIM, K, false>), dim3(items), dim3(SBLOCK), 0, s, p, counts_or_offs, out);
    return hipGetLastError();
}

template <int NDIM, int K> int cand_classes_t() { return SShape<NDIM, K>::NCLS; }

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
using CandFn = hipError_t (*)(const Params&, bool, int*, int*, hipStream_t);
using ClsFn = int (*)();

template <int NDIM> static BinFn pick_bin(int k) { IBTK_LE_DISPATCH(NDIM, k, launch_bin_t) }
template <int NDIM> static InterpFn pick_interp(int k) { IBTK_LE_DISPATCH(NDIM, k, launch_interp_t) }
template <int NDIM> static SpreadFn pick_spread(int k) { IBTK_LE_DISPATCH(NDIM, k, launch_spread_t) }
template <int NDIM> static CandFn pick_cand(int k) { IBTK_LE_DISPATCH(NDIM, k, launch_cand_t) }
template <int NDIM> static ClsFn pick_cls(int k) { IBTK_LE_DISPATCH(NDIM, k, cand_classes_t) }

hipError_t launch_bin(int ndim, int kernel, const Params& p, int n, unsigned* keys, int* vals, hipStream_t s) {
    BinFn f = ndim == 2 ? pick_bin<2>(kernel) : nullptr;  // 3-D: the column sweeps (le_sweep.hip)
    return f ? f(p, n, keys, vals, s) : hipErrorInvalidValue;
}
hipError_t launch_brick_start(const unsigned* keys, int n, int nbricks, int shift, int* bs, hipStream_t s) {
    hipLaunchKernelGGL(k_brick_start, dim3((n + 1 + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, s, keys, n, nbricks, shift,
                       bs);
    return hipGetLastError();
}
hipError_t launch_gather_sorted(int ndim, const Params& p, int n, int* sorted_s, double* sorted_X, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    if (ndim != 2) return hipErrorInvalidValue;  // 3-D: k_gather_col (le_sweep.hip)
    hipLaunchKernelGGL(k_gather_sorted<2>, dim3((n + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, s, p, n, sorted_s,
                       sorted_X);
    return hipGetLastError();
}
hipError_t launch_interp(int ndim, int kernel, const Params& p, int n, hipStream_t s, hipEvent_t ev0,
                         hipEvent_t ev1) {
    InterpFn f = ndim == 2 ? pick_interp<2>(kernel) : nullptr;
    return f ? f(p, n, s, ev0, ev1) : hipErrorInvalidValue;
}
hipError_t launch_cand(int ndim, int kernel, const Params& p, bool write, int* counts_or_offs, int* out, hipStream_t s) {
    CandFn f = ndim == 2 ? pick_cand<2>(kernel) : nullptr;
    return f ? f(p, write, counts_or_offs, out, s) : hipErrorInvalidValue;
}
int cand_classes(int ndim, int kernel) {
    ClsFn f = ndim == 2 ? pick_cls<2>(kernel) : nullptr;
    return f ? f() : 0;
}
hipError_t launch_spread(int ndim, int kernel, const Params& p, hipStream_t s, hipEvent_t ev0, hipEvent_t ev1) {
    SpreadFn f = ndim == 2 ? pick_spread<2>(kernel) : nullptr;
    return f ? f(p, s, ev0, ev1) : hipErrorInvalidValue;
}

}  // namespace ibtk_le
