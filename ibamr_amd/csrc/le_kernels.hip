// le_kernels.hip -- CDNA4 (gfx950) kernels of the Lagrangian-Eulerian coupling
// path: marker binning, brick-tiled interpolation (gather from an LDS-staged
// grid region) and brick-owned spreading (atomics-free, marker-ordered
// accumulation in LDS).  Replaces the l-loops of
// ibtk/src/lagrangian/fortran/lagrangian_interaction{2,3}d.f.m4.
//
// Layout and work decomposition:
//  * Markers are binned by the cell-frame anchor of their stencil ("key cell")
//    into bricks of 8^3 cells (16^2 in 2-D); sort key = brick * 512 + cell.
//  * interp: one workgroup per non-empty brick stages the union stencil region
//    of all its markers, (8 + HI - LO)^3 points per component, from HBM into
//    LDS with coalesced fp64 loads; one thread per (marker, component) sums its
//    W^3 stencil from LDS in the Fortran loop order (bitwise == oracle).
//  * spread: one workgroup owns the 8^3 grid points of a brick for every
//    component: loads u_old into LDS, walks the markers of the 27 neighbouring
//    bricks in canonical (sorted) order, keeps those whose stencil can touch the
//    brick, and one wave per component adds marker after marker, lane = stencil
//    point.  Every grid point therefore receives its contributions in list
//    order, exactly like the Fortran's sequential l-loop: no atomics,
//    deterministic, bitwise == oracle on the same list order.
//  * Workgroups walk bricks grid-stride; the brick -> workgroup map keeps the
//    bricks an XCD works on at one time contiguous (halo reuse in its L2).
#include <hip/hip_runtime.h>

#include "le_internal.h"
#include "le_stencil.h"

namespace ibtk_le {

template <int NDIM> struct BrickT { static constexpr int B = NDIM == 3 ? BRICK3 : BRICK2; };

__device__ __forceinline__ int xcd_brick(int round_base, int G, int wg) {
    // blocks are dealt round-robin over the 8 XCDs: wg % 8 labels an XCD.
    // Give XCD x the contiguous range [x*G/8, (x+1)*G/8) of this round.
    const int per = G >> 3;
    return round_base + (wg & 7) * per + (wg >> 3);
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
        const int k = key_anchor<K>(xo) + p.bg.ilower[d];
        rel[d] = k - p.bg.kmin[d];
        if (rel[d] < 0 || rel[d] >= p.bg.nb[d] * B) out = true;
    }
    unsigned key;
    if (out) {
        key = (unsigned)p.bg.nbricks << p.bg.shift;
    } else {
        unsigned brick = 0, local = 0;
        for (int d = NDIM - 1; d >= 0; --d) {
            brick = brick * (unsigned)p.bg.nb[d] + (unsigned)(rel[d] / B);
            local = local * (unsigned)B + (unsigned)(rel[d] % B);
        }
        key = (brick << p.bg.shift) | local;
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

template <int NDIM, int K>
hipError_t launch_bin_t(const Params& p, int n, unsigned* keys, int* vals, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL((k_bin<NDIM, K>), dim3((n + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, s, p, n, keys, vals);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// interpolation
// ---------------------------------------------------------------------------
template <int NDIM, int K> struct InterpShape {
    using T = KT<K>;
    static constexpr int B = BrickT<NDIM>::B;
    static constexpr int R = B + T::HI - T::LO;  // region edge (points)
    static constexpr int RV = NDIM == 3 ? R * R * R : R * R;
};

template <int NDIM, int K>
__global__ __launch_bounds__(BLOCK) void k_interp(Params p) {
    using T = KT<K>;
    using S = InterpShape<NDIM, K>;
    constexpr int W = T::W, FAM = T::FAM, B = S::B, R = S::R, RV = S::RV;
    extern __shared__ __attribute__((aligned(16))) double lds[];
    const int nc = p.ncomp;
    const int G = gridDim.x;
    for (int round = 0; round < p.bg.nbricks; round += G) {
        const int b = (G & 7) == 0 ? xcd_brick(round, G, blockIdx.x) : round + blockIdx.x;
        if (b >= p.bg.nbricks) continue;
        const int beg = p.brick_start[b], end = p.brick_start[b + 1];
        if (beg == end) continue;
        int bc[3];
        bc[0] = b % p.bg.nb[0];
        bc[1] = (b / p.bg.nb[0]) % p.bg.nb[1];
        bc[2] = NDIM == 3 ? b / (p.bg.nb[0] * p.bg.nb[1]) : 0;
        int r0[3] = {0, 0, 0};
#pragma unroll
        for (int d = 0; d < NDIM; ++d) r0[d] = p.bg.kmin[d] + bc[d] * B + T::LO;

        __syncthreads();  // the previous brick's readers are done with lds
        // Stage the union stencil region of every component.  Consecutive
        // threads walk x, the contiguous (fastest) Fortran index.
        for (int t = threadIdx.x; t < nc * RV; t += BLOCK) {
            const int c = t / RV, q = t - c * RV;
            const CompDesc& cd = p.comp[c];
            const int g0 = r0[0] + q % R;
            const int g1 = r0[1] + (q / R) % R;
            const int g2 = NDIM == 3 ? r0[2] + q / (R * R) : 0;
            bool in = g0 >= cd.lo[0] && g0 <= cd.hi[0] && g1 >= cd.lo[1] && g1 <= cd.hi[1];
            if (NDIM == 3) in = in && g2 >= cd.lo[2] && g2 <= cd.hi[2];
            double v = 0.0;
            if (in) {
                const int64_t off = (int64_t)(g0 - cd.lo[0]) + (int64_t)(g1 - cd.lo[1]) * cd.s1 +
                                    (NDIM == 3 ? (int64_t)(g2 - cd.lo[2]) * cd.s2 : 0);
                v = cd.u[off];
            }
            lds[t] = v;
        }
        __syncthreads();

        const int n = end - beg;
        for (int t = threadIdx.x; t < n * nc; t += BLOCK) {
            const int e = beg + t / nc;
            const int c = t - (t / nc) * nc;
            const CompDesc& cd = p.comp[c];
            const int l = p.sorted_l[e];
            const int s = p.indices ? p.indices[l] : l;
            St<W> st[NDIM];
            bool ok = true;
#pragma unroll
            for (int d = 0; d < NDIM; ++d) {
                const double Xraw = p.X[(int64_t)NDIM * s + d];
                const double Xs = Xraw + (p.Xshift ? p.Xshift[(int64_t)NDIM * l + d] : 0.0);
                stencil1d<K>(Xs, Xraw, cd.xlo[d], p.bg.dx[d], cd.ilower[d], cd.lo[d], cd.hi[d], d == cd.axis, p.K6,
                             st[d]);
                if (st[d].ist <= st[d].isp)
                    ok = ok && (st[d].icl + st[d].ist >= r0[d]) && (st[d].icl + st[d].isp < r0[d] + R);
            }
            if (!ok) {
                atomicOr(p.err, 1);
                continue;
            }
            const double* reg = lds + c * RV;
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
            } else if constexpr (NDIM == 3) {
                const int b0 = st[0].icl - r0[0], b1 = st[1].icl - r0[1], b2 = st[2].icl - r0[2];
#pragma unroll
                for (int i2 = 0; i2 < W; ++i2) {
                    if (i2 < st[2].ist || i2 > st[2].isp) continue;
#pragma unroll
                    for (int i1 = 0; i1 < W; ++i1) {
                        if (i1 < st[1].ist || i1 > st[1].isp) continue;
                        const double* row = reg + (b2 + i2) * (R * R) + (b1 + i1) * R + b0;
                        if constexpr (FAM == 0) {
                            const double wyz = st[1].w[i1] * st[2].w[i2];
#pragma unroll
                            for (int i0 = 0; i0 < W; ++i0) {
                                if (i0 < st[0].ist || i0 > st[0].isp) continue;
                                const double wt = st[0].w[i0] * wyz;
                                acc = acc + wt * row[i0];
                            }
                        } else {
#pragma unroll
                            for (int i0 = 0; i0 < W; ++i0) {
                                if (i0 < st[0].ist || i0 > st[0].isp) continue;
                                acc = acc + st[0].w[i0] * st[1].w[i1] * st[2].w[i2] * row[i0];
                            }
                        }
                    }
                }
            } else {
                const int b0 = st[0].icl - r0[0], b1 = st[1].icl - r0[1];
#pragma unroll
                for (int i1 = 0; i1 < W; ++i1) {
                    if (i1 < st[1].ist || i1 > st[1].isp) continue;
                    const double* row = reg + (b1 + i1) * R + b0;
#pragma unroll
                    for (int i0 = 0; i0 < W; ++i0) {
                        if (i0 < st[0].ist || i0 > st[0].isp) continue;
                        if constexpr (FAM == 0) {
                            const double wt = st[0].w[i0] * st[1].w[i1];
                            acc = acc + wt * row[i0];
                        } else {
                            acc = acc + st[0].w[i0] * st[1].w[i1] * row[i0];
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
        const int l = p.sorted_l[e];
        const int s = p.indices ? p.indices[l] : l;
        for (int c = 0; c < p.ncomp; ++c) p.Qout[(int64_t)p.Q_depth * s + p.comp[c].qcomp] = 0.0;
    }
}

static int grid_for(int nbricks) {
    int dev = 0;
    hipGetDevice(&dev);
    int ncu = 256;
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    long g = (long)ncu * 8;  // resident-ish waves in flight; grid-stride beyond
    if (g > nbricks) g = nbricks;
    if (g >= 8) g &= ~7L;  // multiple of 8 for the XCD remap
    return (int)(g > 0 ? g : 1);
}

template <int NDIM, int K>
hipError_t launch_interp_t(const Params& p, int n, hipStream_t s, hipEvent_t ev0, hipEvent_t ev1) {
    using S = InterpShape<NDIM, K>;
    const size_t lds = (size_t)p.ncomp * S::RV * sizeof(double);
    if (lds > 160 * 1024) return hipErrorInvalidValue;
    if (lds > 64 * 1024)
        hipFuncSetAttribute((const void*)k_interp<NDIM, K>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (ev0) hipEventRecord(ev0, s);
    hipLaunchKernelGGL((k_interp<NDIM, K>), dim3(grid_for(p.bg.nbricks)), dim3(BLOCK), lds, s, p);
    if (ev1) hipEventRecord(ev1, s);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    if (n > 0) hipLaunchKernelGGL(k_interp_outside, dim3(64), dim3(BLOCK), 0, s, p, n);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// spreading
// ---------------------------------------------------------------------------
template <int NDIM, int K> struct SpreadShape {
    using T = KT<K>;
    static constexpr int B = BrickT<NDIM>::B;
    static constexpr int BV = NDIM == 3 ? B * B * B : B * B;
    static constexpr int W = T::W;
    static constexpr int P = NDIM == 3 ? W * W * W : W * W;
    static constexpr int NB = NDIM == 3 ? 27 : 9;
    static constexpr int CH = SPREAD_CH;
    static size_t lds_bytes(int nc) {
        size_t b = 0;
        b += (size_t)nc * BV * sizeof(double);              // acc
        b += (size_t)CH * nc * NDIM * W * sizeof(double);   // candidate weights
        b += (size_t)CH * nc * sizeof(double);              // candidate values
        b += (size_t)CH * nc * NDIM * 3 * sizeof(int);      // candidate stencil info
        b += (size_t)(2 * NB + 1 + 3) * sizeof(int);        // neighbour ranges + misc
        return (b + 15) & ~(size_t)15;
    }
};

template <int NDIM, int K>
__global__ __launch_bounds__(BLOCK) void k_spread(Params p) {
    using T = KT<K>;
    using S = SpreadShape<NDIM, K>;
    constexpr int W = T::W, FAM = T::FAM, LO = T::LO, HI = T::HI;
    constexpr int B = S::B, BV = S::BV, P = S::P, NB = S::NB, CH = S::CH;
    extern __shared__ __attribute__((aligned(16))) double lds[];
    const int nc = p.ncomp;
    double* acc = lds;
    double* cw = acc + nc * BV;
    double* cF = cw + CH * nc * NDIM * W;
    int* cinfo = reinterpret_cast<int*>(cF + CH * nc);
    int* nstart = cinfo + CH * nc * NDIM * 3;
    int* npre = nstart + NB;
    int* misc = npre + NB + 1;
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int G = gridDim.x;

    for (int round = 0; round < p.bg.nbricks; round += G) {
        const int b = (G & 7) == 0 ? xcd_brick(round, G, blockIdx.x) : round + blockIdx.x;
        if (b >= p.bg.nbricks) continue;
        int bc[3];
        bc[0] = b % p.bg.nb[0];
        bc[1] = (b / p.bg.nb[0]) % p.bg.nb[1];
        bc[2] = NDIM == 3 ? b / (p.bg.nb[0] * p.bg.nb[1]) : 0;
        int kb0[3] = {0, 0, 0};
#pragma unroll
        for (int d = 0; d < NDIM; ++d) kb0[d] = p.bg.kmin[d] + bc[d] * B;

        __syncthreads();  // previous brick is fully written back
        if (threadIdx.x < NB) {
            // neighbours in increasing linear brick id: (dz, dy, dx) lexicographic
            const int j = threadIdx.x;
            int off[3];
            off[0] = j % 3 - 1;
            off[1] = (j / 3) % 3 - 1;
            off[2] = NDIM == 3 ? j / 9 - 1 : 0;
            bool valid = true;
            int lin = 0;
            for (int d = NDIM - 1; d >= 0; --d) {
                const int q = bc[d] + off[d];
                valid = valid && q >= 0 && q < p.bg.nb[d];
                lin = lin * p.bg.nb[d] + q;
            }
            const int st = valid ? p.brick_start[lin] : 0;
            const int en = valid ? p.brick_start[lin + 1] : 0;
            nstart[j] = st;
            npre[j + 1] = en - st;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            npre[0] = 0;
            for (int j = 0; j < NB; ++j) npre[j + 1] += npre[j];
        }
        __syncthreads();
        const int total = npre[NB];
        if (total == 0) continue;

        // u_old of the brick's points for every component
        for (int t = threadIdx.x; t < nc * BV; t += BLOCK) {
            const int c = t / BV, q = t - c * BV;
            const CompDesc& cd = p.comp[c];
            const int g0 = kb0[0] + q % B;
            const int g1 = kb0[1] + (q / B) % B;
            const int g2 = NDIM == 3 ? kb0[2] + q / (B * B) : 0;
            bool in = g0 >= cd.lo[0] && g0 <= cd.hi[0] && g1 >= cd.lo[1] && g1 <= cd.hi[1];
            if (NDIM == 3) in = in && g2 >= cd.lo[2] && g2 <= cd.hi[2];
            double v = 0.0;
            if (in) {
                const int64_t o = (int64_t)(g0 - cd.lo[0]) + (int64_t)(g1 - cd.lo[1]) * cd.s1 +
                                  (NDIM == 3 ? (int64_t)(g2 - cd.lo[2]) * cd.s2 : 0);
                v = cd.u[o];
            }
            acc[t] = v;
        }

        for (int base = 0; base < total; base += CH) {
            __syncthreads();  // acc loaded / previous chunk consumed
            if (wave == 0) {
                // filter one chunk of the 27 neighbours' sorted entries, keeping order
                const int e = base + lane;
                bool cand = false;
                int idx = 0;
                int kc[3] = {0, 0, 0};
                if (e < total) {
                    int j = 0;
                    while (npre[j + 1] <= e) ++j;
                    idx = nstart[j] + (e - npre[j]);
                    const unsigned key = p.sorted_key[idx];
                    const unsigned bb = key >> p.bg.shift;
                    unsigned loc = key & ((1u << p.bg.shift) - 1u);
                    unsigned bq = bb;
                    cand = true;
#pragma unroll
                    for (int d = 0; d < NDIM; ++d) {
                        const int bcd = (int)(bq % (unsigned)p.bg.nb[d]);
                        bq /= (unsigned)p.bg.nb[d];
                        const int lcd = (int)(loc % (unsigned)B);
                        loc /= (unsigned)B;
                        kc[d] = p.bg.kmin[d] + bcd * B + lcd;
                        cand = cand && kc[d] >= kb0[d] - HI && kc[d] <= kb0[d] + B - 1 - LO;
                    }
                }
                const unsigned long long mask = __ballot(cand);
                const int pos = __popcll(mask & ((1ull << lane) - 1ull));
                if (lane == 0) misc[0] = __popcll(mask);
                if (cand) {
                    const int l = p.sorted_l[idx];
                    const int s = p.indices ? p.indices[l] : l;
                    double Xraw[3], Xs[3];
#pragma unroll
                    for (int d = 0; d < NDIM; ++d) {
                        Xraw[d] = p.X[(int64_t)NDIM * s + d];
                        Xs[d] = Xraw[d] + (p.Xshift ? p.Xshift[(int64_t)NDIM * l + d] : 0.0);
                    }
                    for (int c = 0; c < nc; ++c) {
                        const CompDesc& cd = p.comp[c];
                        cF[pos * nc + c] = p.Qin[(int64_t)p.Q_depth * s + cd.qcomp];
#pragma unroll
                        for (int d = 0; d < NDIM; ++d) {
                            St<W> st;
                            stencil1d<K>(Xs[d], Xraw[d], cd.xlo[d], p.bg.dx[d], cd.ilower[d], cd.lo[d], cd.hi[d],
                                         d == cd.axis, p.K6, st);
                            // binning invariant: the stencil lies in [key + LO, key + HI]
                            if (st.ist <= st.isp &&
                                (st.icl + st.ist < kc[d] + LO || st.icl + st.isp > kc[d] + HI))
                                atomicOr(p.err, 2);
                            int* inf = cinfo + ((pos * nc + c) * NDIM + d) * 3;
                            inf[0] = st.icl;
                            inf[1] = st.ist;
                            inf[2] = st.isp;
                            double* wd = cw + ((pos * nc + c) * NDIM + d) * W;
#pragma unroll
                            for (int i = 0; i < W; ++i) {
                                // closed form: wz = w2/(dx0*dx1*dx2) (f.m4:1486), 2-D wy = w1/(dx0*dx1)
                                wd[i] = (FAM == 0 && d == NDIM - 1) ? st.w[i] / p.h3 : st.w[i];
                            }
                        }
                    }
                }
            }
            __syncthreads();
            const int ncand = misc[0];
            if (wave < nc) {
                const int c = wave;
                double* ac = acc + c * BV;
                for (int ci = 0; ci < ncand; ++ci) {
                    const int* inf = cinfo + (ci * nc + c) * NDIM * 3;
                    const double* w = cw + (ci * nc + c) * NDIM * W;
                    const double F = cF[ci * nc + c];
                    for (int q = lane; q < P; q += 64) {
                        int ii[3];
                        ii[0] = q % W;
                        ii[1] = (q / W) % W;
                        ii[2] = NDIM == 3 ? q / (W * W) : 0;
                        bool ok = true;
                        int li = 0, mul = 1;
#pragma unroll
                        for (int d = 0; d < NDIM; ++d) {
                            ok = ok && ii[d] >= inf[d * 3 + 1] && ii[d] <= inf[d * 3 + 2];
                            const int lc = inf[d * 3] + ii[d] - kb0[d];
                            ok = ok && lc >= 0 && lc < B;
                            li += lc * mul;
                            mul *= B;
                        }
                        if (!ok) continue;
                        double contrib;
                        if constexpr (FAM == 3) {
                            contrib = F / p.h3;  // f.m4:170-171
                        } else if constexpr (FAM == 0) {
                            if constexpr (NDIM == 3) {
                                const double wt = w[ii[0]] * (w[W + ii[1]] * w[2 * W + ii[2]]);
                                contrib = wt * F;
                            } else {
                                const double wt = w[ii[0]] * w[W + ii[1]];
                                contrib = wt * F;
                            }
                        } else {
                            if constexpr (NDIM == 3)
                                contrib = w[ii[0]] * w[W + ii[1]] * w[2 * W + ii[2]] * F / p.h3;
                            else
                                contrib = w[ii[0]] * w[W + ii[1]] * F / p.h3;
                        }
                        ac[li] = ac[li] + contrib;
                    }
                }
            }
        }
        __syncthreads();
        for (int t = threadIdx.x; t < nc * BV; t += BLOCK) {
            const int c = t / BV, q = t - c * BV;
            const CompDesc& cd = p.comp[c];
            const int g0 = kb0[0] + q % B;
            const int g1 = kb0[1] + (q / B) % B;
            const int g2 = NDIM == 3 ? kb0[2] + q / (B * B) : 0;
            bool in = g0 >= cd.lo[0] && g0 <= cd.hi[0] && g1 >= cd.lo[1] && g1 <= cd.hi[1];
            if (NDIM == 3) in = in && g2 >= cd.lo[2] && g2 <= cd.hi[2];
            if (in) {
                const int64_t o = (int64_t)(g0 - cd.lo[0]) + (int64_t)(g1 - cd.lo[1]) * cd.s1 +
                                  (NDIM == 3 ? (int64_t)(g2 - cd.lo[2]) * cd.s2 : 0);
                cd.u[o] = acc[t];
            }
        }
    }
}

template <int NDIM, int K>
hipError_t launch_spread_t(const Params& p, hipStream_t s, hipEvent_t ev0, hipEvent_t ev1) {
    using S = SpreadShape<NDIM, K>;
    const size_t lds = S::lds_bytes(p.ncomp);
    if (lds > 160 * 1024) return hipErrorInvalidValue;
    if (lds > 64 * 1024)
        hipFuncSetAttribute((const void*)k_spread<NDIM, K>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (ev0) hipEventRecord(ev0, s);
    hipLaunchKernelGGL((k_spread<NDIM, K>), dim3(grid_for(p.bg.nbricks)), dim3(BLOCK), lds, s, p);
    if (ev1) hipEventRecord(ev1, s);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// diagnostics: mark every array point some listed stencil touches (after
// clipping), for the exact algorithmic-byte count |S_a| of the roofline.
// ---------------------------------------------------------------------------
template <int NDIM, int K>
__global__ __launch_bounds__(BLOCK) void k_mark(Params p, int n, unsigned char* m0, unsigned char* m1,
                                                unsigned char* m2, unsigned char* m3) {
    constexpr int W = KT<K>::W;
    const int e = blockIdx.x * BLOCK + threadIdx.x;
    if (e >= n) return;
    const int s = p.indices ? p.indices[e] : e;
    unsigned char* masks[4] = {m0, m1, m2, m3};
    for (int c = 0; c < p.ncomp; ++c) {
        const CompDesc& cd = p.comp[c];
        St<W> st[NDIM];
        for (int d = 0; d < NDIM; ++d) {
            const double Xraw = p.X[(int64_t)NDIM * s + d];
            const double Xs = Xraw + (p.Xshift ? p.Xshift[(int64_t)NDIM * e + d] : 0.0);
            stencil1d<K>(Xs, Xraw, cd.xlo[d], p.bg.dx[d], cd.ilower[d], cd.lo[d], cd.hi[d], d == cd.axis, p.K6,
                         st[d]);
        }
        for (int i2 = (NDIM == 3 ? st[NDIM - 1].ist : 0); i2 <= (NDIM == 3 ? st[NDIM - 1].isp : 0); ++i2)
            for (int i1 = st[1].ist; i1 <= st[1].isp; ++i1)
                for (int i0 = st[0].ist; i0 <= st[0].isp; ++i0) {
                    const int g0 = st[0].icl + i0, g1 = st[1].icl + i1;
                    const int g2 = NDIM == 3 ? st[NDIM - 1].icl + i2 : 0;
                    const int64_t o = (int64_t)(g0 - cd.lo[0]) + (int64_t)(g1 - cd.lo[1]) * cd.s1 +
                                      (NDIM == 3 ? (int64_t)(g2 - cd.lo[2]) * cd.s2 : 0);
                    masks[c][o] = 1;  // idempotent, benign race
                }
    }
}

template <int NDIM, int K>
hipError_t launch_mark_t(const Params& p, int n, unsigned char** masks, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL((k_mark<NDIM, K>), dim3((n + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, s, p, n, masks[0], masks[1],
                       masks[2], masks[3]);
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
using MarkFn = hipError_t (*)(const Params&, int, unsigned char**, hipStream_t);
template <int NDIM> static MarkFn pick_mark(int k) { IBTK_LE_DISPATCH(NDIM, k, launch_mark_t) }

hipError_t launch_bin(int ndim, int kernel, const Params& p, int n, unsigned* keys, int* vals, hipStream_t s) {
    BinFn f = ndim == 3 ? pick_bin<3>(kernel) : pick_bin<2>(kernel);
    return f ? f(p, n, keys, vals, s) : hipErrorInvalidValue;
}
hipError_t launch_brick_start(const unsigned* keys, int n, int nbricks, int shift, int* bs, hipStream_t s) {
    hipLaunchKernelGGL(k_brick_start, dim3((n + 1 + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, s, keys, n, nbricks, shift,
                       bs);
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

hipError_t launch_mark(int ndim, int kernel, const Params& p, int n, unsigned char** masks, hipStream_t s) {
    MarkFn f = ndim == 3 ? pick_mark<3>(kernel) : pick_mark<2>(kernel);
    return f ? f(p, n, masks, s) : hipErrorInvalidValue;
}

// ---------------------------------------------------------------------------
// periodic ghost fill / ghost-region fold / ghost zeroing
// ---------------------------------------------------------------------------
// The ghost region of dim d (d = 0..NDIM-1): dims > d interior, dim d outside
// the interior, dims < d anything in the ghost box.
__device__ __forceinline__ bool ghost_point(const GhostDesc& g, int ndim, int dreg, int64_t t, int* pt) {
    int64_t rem = t;
    int ext[3];
    for (int d = 0; d < ndim; ++d) {
        if (d < dreg) ext[d] = g.hi[d] - g.lo[d] + 1;
        else if (d == dreg) ext[d] = (g.ilo[d] - g.lo[d]) + (g.hi[d] - g.ihi[d]);
        else ext[d] = g.ihi[d] - g.ilo[d] + 1;
    }
    for (int d = 0; d < ndim; ++d) {
        const int q = (int)(rem % ext[d]);
        rem /= ext[d];
        if (d < dreg) pt[d] = g.lo[d] + q;
        else if (d == dreg) {
            const int nlo = g.ilo[d] - g.lo[d];
            pt[d] = q < nlo ? g.lo[d] + q : g.ihi[d] + 1 + (q - nlo);
        } else pt[d] = g.ilo[d] + q;
    }
    return rem == 0;
}

__device__ __forceinline__ int64_t goff(const GhostDesc& g, int ndim, const int* pt) {
    int64_t o = pt[0] - g.lo[0];
    if (ndim > 1) o += (int64_t)(pt[1] - g.lo[1]) * g.s1;
    if (ndim > 2) o += (int64_t)(pt[2] - g.lo[2]) * g.s2;
    return o;
}

__device__ __forceinline__ int wrap(int i, int lo, int n) {
    int r = (i - lo) % n;
    if (r < 0) r += n;
    return lo + r;
}

// mode 0: fill (ghost <- periodic interior, all dims wrapped at once)
// mode 1: fold dim dreg (interior-in-dreg point += ghost point), one source per destination
// mode 2: zero
__global__ __launch_bounds__(BLOCK) void k_ghost(GhostDesc g, int ndim, int dreg, int mode, int64_t count, int p0,
                                                  int p1, int p2) {
    const int64_t t = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (t >= count) return;
    int pt[3] = {0, 0, 0};
    if (!ghost_point(g, ndim, dreg, t, pt)) return;
    const int per[3] = {p0, p1, p2};
    if (mode == 2) {
        g.u[goff(g, ndim, pt)] = 0.0;
        return;
    }
    if (mode == 0) {
        int src[3] = {pt[0], pt[1], pt[2]};
        for (int d = 0; d < ndim; ++d) {
            if (src[d] < g.ilo[d] || src[d] > g.ihi[d]) {
                if (!per[d]) return;
                src[d] = wrap(src[d], g.ilo[d], g.ihi[d] - g.ilo[d] + 1);
            }
        }
        g.u[goff(g, ndim, pt)] = g.u[goff(g, ndim, src)];
        return;
    }
    // fold along dreg only
    if (!per[dreg]) return;
    int dst[3] = {pt[0], pt[1], pt[2]};
    dst[dreg] = wrap(pt[dreg], g.ilo[dreg], g.ihi[dreg] - g.ilo[dreg] + 1);
    const int64_t os = goff(g, ndim, pt), od = goff(g, ndim, dst);
    g.u[od] = g.u[od] + g.u[os];
}

static int64_t ghost_count(const GhostDesc& g, int ndim, int dreg) {
    int64_t c = 1;
    for (int d = 0; d < ndim; ++d) {
        if (d < dreg) c *= g.hi[d] - g.lo[d] + 1;
        else if (d == dreg) c *= (g.ilo[d] - g.lo[d]) + (g.hi[d] - g.ihi[d]);
        else c *= g.ihi[d] - g.ilo[d] + 1;
    }
    return c;
}

static hipError_t ghost_pass(const GhostDesc& g, int ndim, int dreg, int mode, const int* per, hipStream_t s) {
    const int64_t cnt = ghost_count(g, ndim, dreg);
    if (cnt <= 0) return hipSuccess;
    const int64_t nb = (cnt + BLOCK - 1) / BLOCK;
    hipLaunchKernelGGL(k_ghost, dim3((unsigned)nb), dim3(BLOCK), 0, s, g, ndim, dreg, mode, cnt, per[0], per[1],
                       ndim > 2 ? per[2] : 0);
    return hipGetLastError();
}

hipError_t launch_fill_periodic(int ndim, const GhostDesc& g, const int* periodic, hipStream_t s) {
    for (int d = 0; d < ndim; ++d) {
        hipError_t e = ghost_pass(g, ndim, d, 0, periodic, s);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}
hipError_t launch_fold_periodic(int ndim, const GhostDesc& g, const int* periodic, hipStream_t s) {
    // slowest dim first: a point that is ghost in several dims is carried into
    // the interior one dim at a time, each step with one source per destination
    for (int d = ndim - 1; d >= 0; --d) {
        hipError_t e = ghost_pass(g, ndim, d, 1, periodic, s);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}
hipError_t launch_zero_ghosts(int ndim, const GhostDesc& g, hipStream_t s) {
    const int per[3] = {1, 1, 1};
    for (int d = 0; d < ndim; ++d) {
        hipError_t e = ghost_pass(g, ndim, d, 2, per, s);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

// ---------------------------------------------------------------------------
// periodic index lists (LIndexSetData::cacheLocalIndices for one periodic patch)
// ---------------------------------------------------------------------------
__device__ __forceinline__ void cell_index(const ImageDesc& d, const double* X, int* c) {
    // IndexUtilities::getCellIndex, IndexUtilities-inl.h:66-89
    for (int k = 0; k < d.ndim; ++k) {
        const double dl = X[k] - d.xlo[k], du = X[k] - d.xup[k];
        if (fabs(dl) <= fabs(du)) c[k] = d.ilo[k] + (int)floor(dl / d.dx[k]);
        else c[k] = d.ihi[k] + (int)floor(du / d.dx[k]) + 1;
    }
}

__device__ __forceinline__ int image_walk(const ImageDesc& d, const double* X, int* idx_out, double* xs_out,
                                          int base, int capacity, int s) {
    int c[3] = {0, 0, 0};
    cell_index(d, X, c);
    for (int k = 0; k < d.ndim; ++k)
        if (c[k] < d.ilo[k] || c[k] > d.ihi[k]) return 0;  // not owned by this patch
    int cnt = 0;
    const int nimg = d.ndim == 3 ? 27 : 9;
    for (int j = 0; j < nimg; ++j) {
        // j = 13 (3-D) / 4 (2-D) is the unshifted entry; emit it first
        const int jj = j == 0 ? (nimg / 2) : (j <= nimg / 2 ? j - 1 : j);
        int sh[3] = {jj % 3 - 1, (jj / 3) % 3 - 1, d.ndim == 3 ? jj / 9 - 1 : 0};
        bool ok = true;
        for (int k = 0; k < d.ndim; ++k) {
            if (sh[k] != 0 && !d.periodic[k]) ok = false;
            const int n = d.ihi[k] - d.ilo[k] + 1;
            const int ci = c[k] + sh[k] * n;
            ok = ok && ci >= d.ilo[k] - d.ghost && ci <= d.ihi[k] + d.ghost;
        }
        if (!ok) continue;
        if (idx_out && base + cnt < capacity) {
            idx_out[base + cnt] = s;
            for (int k = 0; k < d.ndim; ++k) {
                const int n = d.ihi[k] - d.ilo[k] + 1;
                // LIndexSetData.cpp:141: static_cast<double>(offset[d]) * dx[d]
                xs_out[(int64_t)d.ndim * (base + cnt) + k] = (double)(sh[k] * n) * d.dx[k];
            }
        }
        ++cnt;
    }
    return cnt;
}

__global__ __launch_bounds__(BLOCK) void k_image_count(ImageDesc d, const double* X, int n, int* counts) {
    const int s = blockIdx.x * BLOCK + threadIdx.x;
    if (s >= n) return;
    counts[s] = image_walk(d, X + (int64_t)d.ndim * s, nullptr, nullptr, 0, 0, s);
}
__global__ __launch_bounds__(BLOCK) void k_image_write(ImageDesc d, const double* X, int n, const int* offsets,
                                                        int* idx, double* xs, int capacity) {
    const int s = blockIdx.x * BLOCK + threadIdx.x;
    if (s >= n) return;
    image_walk(d, X + (int64_t)d.ndim * s, idx, xs, offsets[s], capacity, s);
}

hipError_t launch_image_count(const ImageDesc& d, const double* X, int n, int* counts, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_image_count, dim3((n + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, s, d, X, n, counts);
    return hipGetLastError();
}
hipError_t launch_image_write(const ImageDesc& d, const double* X, int n, const int* offsets, int* idx,
                              double* xshift, int capacity, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_image_write, dim3((n + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, s, d, X, n, offsets, idx,
                       xshift, capacity);
    return hipGetLastError();
}

}  // namespace ibtk_le
