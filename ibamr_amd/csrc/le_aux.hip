// le_aux.hip -- auxiliary device kernels of the LE coupling path: stencil
// marking (roofline byte counts), periodic ghost fill / ghost-region fold, and
// the periodic / box index lists (LIndexSetData::cacheLocalIndices,
// LEInteractor::buildLocalIndices for one patch).  The hot path is le_hot.hip.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>

#include "le_internal.h"
#include "le_stencil.h"

namespace ibtk_le {

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

using MarkFn = hipError_t (*)(const Params&, int, unsigned char**, hipStream_t);
template <int NDIM> static MarkFn pick_mark(int k) { IBTK_LE_DISPATCH(NDIM, k, launch_mark_t) }

hipError_t launch_mark(int ndim, int kernel, const Params& p, int n, unsigned char** masks, hipStream_t s) {
    MarkFn f = ndim == 3 ? pick_mark<3>(kernel) : pick_mark<2>(kernel);
    return f ? f(p, n, masks, s) : hipErrorInvalidValue;
}

// ---------------------------------------------------------------------------
// periodic ghost fill / ghost-region fold / ghost zeroing
// ---------------------------------------------------------------------------
// The ghost region of dim d (d = 0..NDIM-1): dims > d interior, dim d outside
// the interior, dims < d anything in the ghost box.
// Extents of pass dreg: dims below dreg over the whole ghost box, dim dreg over
// its ghost layers only, dims above over the interior if periodic (their ghosts
// are another pass's) and over the whole ghost box if not (their ghosts are
// physical: the fill copies them from the periodic image, which the physical
// fill has set before; the fold carries them to the image, for the physical
// fold that follows).
__device__ __host__ __forceinline__ bool full_dim(int d, int dreg, const int* per) { return d < dreg || !per[d]; }
__device__ __host__ __forceinline__ void ghost_ext(const GhostDesc& g, int ndim, int dreg, const int* per, int* ext) {
    for (int d = 0; d < 3; ++d) {
        if (d >= ndim) ext[d] = 1;
        else if (d == dreg) ext[d] = (g.ilo[d] - g.lo[d]) + (g.hi[d] - g.ihi[d]);
        else if (full_dim(d, dreg, per)) ext[d] = g.hi[d] - g.lo[d] + 1;
        else ext[d] = g.ihi[d] - g.ilo[d] + 1;
    }
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

// One pass over the ghost points of dim dreg of up to GSET arrays (blockIdx.z =
// array): dims 0 and 1 flattened over x blocks (one 32-bit division per
// thread), dim 2 over blockIdx.y.
// mode 0: fill (ghost <- its image with every periodic dim wrapped at once)
// mode 1: fold dim dreg (interior-in-dreg point += ghost point), one source per destination
// mode 2: zero
__device__ __forceinline__ void ghost_point(const GhostDesc& g, int ndim, int dreg, int mode, const int* per,
                                            const int* pt) {
    if (mode == 2) {
        g.u[goff(g, ndim, pt)] = 0.0;
        return;
    }
    if (mode == 0) {
        int src[3] = {pt[0], pt[1], pt[2]};
        bool moved = false;  // wrapped in some periodic dim (a non-periodic ghost coordinate is kept)
        for (int d = 0; d < ndim; ++d) {
            if (per[d] && (src[d] < g.ilo[d] || src[d] > g.ihi[d])) {
                src[d] = wrap(src[d], g.ilo[d], g.ihi[d] - g.ilo[d] + 1);
                moved = true;
            }
        }
        if (moved) g.u[goff(g, ndim, pt)] = g.u[goff(g, ndim, src)];
        return;
    }
    // fold along dreg only
    if (!per[dreg]) return;
    int dst[3] = {pt[0], pt[1], pt[2]};
    dst[dreg] = wrap(pt[dreg], g.ilo[dreg], g.ihi[dreg] - g.ilo[dreg] + 1);
    const int64_t os = goff(g, ndim, pt), od = goff(g, ndim, dst);
    g.u[od] = g.u[od] + g.u[os];
}

// VX points of dim 0 per thread (q0 + v ex0: each instruction coalesced) in the
// passes where dim 0 is long (dreg > 0: its whole ghost box or interior): VX
// independent loads in flight per thread instead of one.
template <int VX>
__global__ __launch_bounds__(BLOCK) void k_ghost(GhostSet gs, int ndim, int dreg, int mode, int p0, int p1, int p2) {
    const GhostDesc& g = gs.g[blockIdx.z];
    const int per[3] = {p0, p1, p2};
    int ext[3];
    ghost_ext(g, ndim, dreg, per, ext);
    const unsigned ex0 = (unsigned)(ext[0] + VX - 1) / VX;  // thread columns along dim 0
    const unsigned t = blockIdx.x * BLOCK + threadIdx.x;
    if (t >= ex0 * (unsigned)ext[1] || (int)blockIdx.y >= ext[2]) return;
    const int q0 = (int)(t % ex0), q[2] = {(int)(t / ex0), (int)blockIdx.y};  // points q0 + v ex0 (coalesced per v)
    int base[3] = {0, 0, 0};
    for (int d = 0; d < ndim; ++d) {
        const int qd = d == 0 ? q0 : q[d - 1];
        if (d == dreg) {
            const int nlo = g.ilo[d] - g.lo[d];
            base[d] = qd < nlo ? g.lo[d] + qd : g.ihi[d] + 1 + (qd - nlo);
        } else if (full_dim(d, dreg, per)) base[d] = g.lo[d] + qd;
        else base[d] = g.ilo[d] + qd;
    }
#pragma unroll
    for (int v = 0; v < VX; ++v) {
        if (q0 + v * (int)ex0 >= ext[0]) break;
        const int pt[3] = {base[0] + v * (int)ex0, base[1], base[2]};  // dreg > 0 when VX > 1: dim 0 is contiguous
        ghost_point(g, ndim, dreg, mode, per, pt);
    }
}

static hipError_t ghost_pass(const GhostDesc* gds, int n, int ndim, int dreg, int mode, const int* per,
                             hipStream_t s) {
    for (int first = 0; first < n; first += GSET) {
        GhostSet gs;
        std::memset(&gs, 0, sizeof(gs));
        const int cnt = std::min(GSET, n - first);
        long long m01 = 0;
        int m2 = 0;
        for (int i = 0; i < cnt; ++i) {
            gs.g[i] = gds[first + i];
            int ext[3];
            ghost_ext(gs.g[i], ndim, dreg, per, ext);
            m01 = std::max(m01, (long long)ext[0] * ext[1]);
            m2 = std::max(m2, ext[2]);
        }
        if (m01 <= 0 || m2 <= 0) continue;
        if (m01 >= (1LL << 32) || m2 > 65535) return hipErrorInvalidValue;
        if (dreg > 0) {  // dim 0 long and contiguous: 4 points a thread
            long long mv = 0;
            for (int i = 0; i < cnt; ++i) {
                int ext[3];
                ghost_ext(gs.g[i], ndim, dreg, per, ext);
                mv = std::max(mv, (long long)((ext[0] + 3) / 4) * ext[1]);
            }
            hipLaunchKernelGGL(k_ghost<4>, dim3((unsigned)((mv + BLOCK - 1) / BLOCK), (unsigned)m2, (unsigned)cnt),
                               dim3(BLOCK), 0, s, gs, ndim, dreg, mode, per[0], per[1], ndim > 2 ? per[2] : 0);
        } else {
            hipLaunchKernelGGL(k_ghost<1>, dim3((unsigned)((m01 + BLOCK - 1) / BLOCK), (unsigned)m2, (unsigned)cnt),
                               dim3(BLOCK), 0, s, gs, ndim, dreg, mode, per[0], per[1], ndim > 2 ? per[2] : 0);
        }
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

// After the physical fill when some dims are not periodic (their ghost layers
// are copied from the periodic image like any other point).
hipError_t launch_fill_periodic(int ndim, const GhostDesc* g, int n, const int* periodic, hipStream_t s) {
    for (int d = 0; d < ndim; ++d) {
        hipError_t e = ghost_pass(g, n, ndim, d, 0, periodic, s);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}
hipError_t launch_fold_periodic(int ndim, const GhostDesc* g, int n, const int* periodic, hipStream_t s) {
    // slowest dim first: a point that is ghost in several dims is carried into
    // the interior one dim at a time, each step with one source per destination
    for (int d = ndim - 1; d >= 0; --d) {
        hipError_t e = ghost_pass(g, n, ndim, d, 1, periodic, s);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}
hipError_t launch_zero_ghosts(int ndim, const GhostDesc* g, int n, hipStream_t s) {
    const int per[3] = {1, 1, 1};
    for (int d = 0; d < ndim; ++d) {
        hipError_t e = ghost_pass(g, n, ndim, d, 2, per, s);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

// ---------------------------------------------------------------------------
// level ghost fill: the RefineSchedule::fillData of LDataManager.cpp:748-751 on
// a level of equal patches tiling a box.  Pass dreg covers the ghost layers of
// dim dreg, the whole ghost extent of the dims below it and the unique points
// of the dims above (the k_ghost regions): every ghost point once.  A point's
// source is the patch owning its (wrapped) cell, at the same global index.
// blockIdx.z = patch * ncomp + array; arrays[patch * ncomp + array] (depth
// slices of a cell array are consecutive arrays of one allocation).
// ---------------------------------------------------------------------------
template <int VX>
__global__ __launch_bounds__(BLOCK) void k_level_fill(LevelTiling t, int dreg, const int* tile_of_patch,
                                                      const int* patch_of_tile, double* const* arrays, int depth) {
    // The source of a ghost point is the neighbouring tile in direction dir (per dim
    // -1, 0, +1) at local index li - dir n: the 27 neighbours' arrays are looked up
    // once per workgroup (the tiles are equal, so a ghost layer no wider than a
    // patch reaches only them; wrapped in the periodic dims, none across a
    // physical boundary -- left to the boundary operators).  VX points of dim 0
    // per thread (q0 + v ex0) where dim 0 is long (dreg > 0).
    const int q = blockIdx.z / t.ncomp, a = blockIdx.z - q * t.ncomp;
    __shared__ const double* nbr[27];
    if (threadIdx.x < 27) {
        const int tile = tile_of_patch[q];
        const int tc[3] = {tile % t.ntile[0], (tile / t.ntile[0]) % t.ntile[1], tile / (t.ntile[0] * t.ntile[1])};
        const int dir[3] = {(int)threadIdx.x % 3 - 1, ((int)threadIdx.x / 3) % 3 - 1, (int)threadIdx.x / 9 - 1};
        int nt[3];
        bool ok = true;
        for (int d = 0; d < 3; ++d) {
            nt[d] = tc[d] + dir[d];
            if (nt[d] < 0 || nt[d] >= t.ntile[d]) {
                if (!t.periodic[d]) ok = false;
                nt[d] = (nt[d] + t.ntile[d]) % t.ntile[d];
            }
        }
        const int sq = ok ? patch_of_tile[nt[0] + t.ntile[0] * (nt[1] + t.ntile[1] * nt[2])] : -1;
        nbr[threadIdx.x] = sq >= 0 ? arrays[(size_t)sq * t.ncomp + a] : nullptr;
    }
    __syncthreads();
    int ext[3];
    for (int d = 0; d < 3; ++d) ext[d] = t.n[d] + 2 * t.g + ((t.side && d == a) ? 1 : 0);  // array extent
    int rx[3];  // region extents of this pass: ghost layers in dreg, all below it, unique points above
    for (int d = 0; d < 3; ++d) rx[d] = d < dreg ? ext[d] : (d == dreg ? ext[d] - t.n[d] : t.n[d]);
    const unsigned ex0 = (unsigned)(rx[0] + VX - 1) / VX;
    const unsigned tid = blockIdx.x * BLOCK + threadIdx.x;
    if (tid >= ex0 * (unsigned)rx[1] || (int)blockIdx.y >= rx[2]) return;
    const int q0 = (int)(tid % ex0), r1 = (int)(tid / ex0), r2 = (int)blockIdx.y;
    const int64_t vol = (int64_t)ext[0] * ext[1] * ext[2];
    double* dst = arrays[(size_t)q * t.ncomp + a];
#pragma unroll
    for (int v = 0; v < VX; ++v) {
        const int r[3] = {q0 + v * (int)ex0, r1, r2};
        if (r[0] >= rx[0]) break;
        int li[3], sl[3], k = 0, mul = 1;
        for (int d = 0; d < 3; ++d) {
            if (d < dreg) li[d] = r[d];
            else if (d == dreg) li[d] = r[d] < t.g ? r[d] : t.g + t.n[d] + (r[d] - t.g);
            else li[d] = t.g + r[d];
            const int dir = li[d] < t.g ? -1 : (li[d] >= t.g + t.n[d] ? 1 : 0);
            sl[d] = li[d] - dir * t.n[d];
            k += (dir + 1) * mul;
            mul *= 3;
        }
        const double* src = nbr[k];
        if (!src) continue;
        const int64_t di = (int64_t)li[0] + (int64_t)ext[0] * (li[1] + (int64_t)ext[1] * li[2]);
        const int64_t si = (int64_t)sl[0] + (int64_t)ext[0] * (sl[1] + (int64_t)ext[1] * sl[2]);
        for (int j = 0; j < depth; ++j) dst[j * vol + di] = src[j * vol + si];
    }
}

// every element of narr arrays := 0 (array i: count[i] doubles, 16-byte aligned
// when count is even), blockIdx.y = array: one launch for a level's patch arrays
__global__ __launch_bounds__(BLOCK) void k_level_zero(double* const* arrays, const long long* count) {
    double* a = arrays[blockIdx.y];
    const long long n = count[blockIdx.y];
    const bool vec = (reinterpret_cast<uintptr_t>(a) & 15) == 0;
    const long long stride = (long long)gridDim.x * BLOCK;
    if (vec) {
        double2* a2 = reinterpret_cast<double2*>(a);
        for (long long i = (long long)blockIdx.x * BLOCK + threadIdx.x; i < n / 2; i += stride) a2[i] = double2{0.0, 0.0};
        if ((n & 1) && blockIdx.x == 0 && threadIdx.x == 0) a[n - 1] = 0.0;
    } else {
        for (long long i = (long long)blockIdx.x * BLOCK + threadIdx.x; i < n; i += stride) a[i] = 0.0;
    }
}
hipError_t launch_level_zero(double* const* arrays, const long long* count, int narr, long long max_count,
                             hipStream_t s) {
    if (narr <= 0 || max_count <= 0) return hipSuccess;
    const long long want = (max_count / 2 + BLOCK - 1) / BLOCK;
    const int gx = (int)std::max(1LL, std::min(want, 64LL));
    hipLaunchKernelGGL(k_level_zero, dim3(gx, narr), dim3(BLOCK), 0, s, arrays, count);
    return hipGetLastError();
}

hipError_t launch_level_fill(const LevelTiling& t, int npatch, const int* tile_of_patch, const int* patch_of_tile,
                             double* const* arrays, int depth, hipStream_t s) {
    for (int dreg = 0; dreg < 3; ++dreg) {
        long long m01 = 0;
        int m2 = 0;
        for (int a = 0; a < t.ncomp; ++a) {
            int rx[3];
            for (int d = 0; d < 3; ++d) {
                const int ext = t.n[d] + 2 * t.g + ((t.side && d == a) ? 1 : 0);
                rx[d] = d < dreg ? ext : (d == dreg ? ext - t.n[d] : t.n[d]);
            }
            m01 = std::max(m01, (long long)rx[0] * rx[1]);
            m2 = std::max(m2, rx[2]);
        }
        if (m01 <= 0 || m2 <= 0) continue;
        const long long nz = (long long)npatch * t.ncomp;
        if (m01 >= (1LL << 32) || m2 > 65535 || nz > 65535) return hipErrorInvalidValue;
        if (dreg > 0) {  // dim 0 long: 4 points a thread
            long long mv = 0;
            for (int a = 0; a < t.ncomp; ++a) {
                const int ext0 = t.n[0] + 2 * t.g + ((t.side && a == 0) ? 1 : 0);
                const int ext1 = t.n[1] + 2 * t.g + ((t.side && a == 1) ? 1 : 0);
                const int rx1 = dreg == 1 ? ext1 - t.n[1] : ext1;
                mv = std::max(mv, (long long)((ext0 + 3) / 4) * rx1);
            }
            hipLaunchKernelGGL(k_level_fill<4>, dim3((unsigned)((mv + BLOCK - 1) / BLOCK), (unsigned)m2, (unsigned)nz),
                               dim3(BLOCK), 0, s, t, dreg, tile_of_patch, patch_of_tile, arrays, depth);
        } else {
            hipLaunchKernelGGL(k_level_fill<1>, dim3((unsigned)((m01 + BLOCK - 1) / BLOCK), (unsigned)m2, (unsigned)nz),
                               dim3(BLOCK), 0, s, t, dreg, tile_of_patch, patch_of_tile, arrays, depth);
        }
        hipError_t e = hipGetLastError();
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
                                          unsigned* key_out, int* cell_out, int base, int capacity, int s) {
    int c[3] = {0, 0, 0};
    cell_index(d, X, c);
    if (d.filter) {  // LEInteractor.cpp:3129-3137: keep markers whose cell is in the box
        for (int k = 0; k < d.ndim; ++k)
            if (c[k] < d.flo[k] || c[k] > d.fhi[k]) return 0;
        if (idx_out && base < capacity) {
            idx_out[base] = s;
            if (xs_out)
                for (int k = 0; k < d.ndim; ++k) xs_out[(int64_t)d.ndim * base + k] = 0.0;
        }
        return 1;
    }
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
        // the image's cell: in the patch box (interior entry) or a ghost cell
        bool interior = true, insub = true;
        unsigned key = 0, stride = 1;
        for (int k = 0; k < d.ndim; ++k) {
            const int n = d.ihi[k] - d.ilo[k] + 1;
            const int ci = c[k] + sh[k] * n;
            interior = interior && ci >= d.ilo[k] && ci <= d.ihi[k];
            insub = insub && ci >= d.slo[k] && ci <= d.shi[k];
            key += (unsigned)(ci - (d.ilo[k] - d.ghost)) * stride;  // ghost-box linear index, x fastest
            stride *= (unsigned)(n + 2 * d.ghost);
        }
        if ((d.which == 1 && !interior) || (d.which == 2 && interior)) continue;
        if (d.sub && !insub) continue;  // LEInteractor.cpp:3075: if (!box.contains(i)) continue
        if (idx_out && base + cnt < capacity) {
            idx_out[base + cnt] = s;
            if (key_out) key_out[base + cnt] = key;
            if (cell_out)
                for (int k = 0; k < d.ndim; ++k)
                    cell_out[(int64_t)d.ndim * (base + cnt) + k] = c[k] + sh[k] * (d.ihi[k] - d.ilo[k] + 1);
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
    counts[s] = image_walk(d, X + (int64_t)d.ndim * s, nullptr, nullptr, nullptr, nullptr, 0, 0, s);
}
__global__ __launch_bounds__(BLOCK) void k_image_write(ImageDesc d, const double* X, int n, const int* offsets,
                                                        int* idx, double* xs, unsigned* cellkey, int* cells,
                                                        int capacity) {
    const int s = blockIdx.x * BLOCK + threadIdx.x;
    if (s >= n) return;
    image_walk(d, X + (int64_t)d.ndim * s, idx, xs, cellkey, cells, offsets[s], capacity, s);
}

// ---------------------------------------------------------------------------
// reference-ordered lists: LIndexSetData::cacheLocalIndices walks the ghost
// box's cells in iteration order and, in each cell, its LNodeSet -- sorted by
// Lagrangian index and uniqued at redistribution (LDataManager.cpp:1487-1493).
// Two stable radix passes (Lagrangian index, then cell) give that order.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(BLOCK) void k_iota(int* v, int n) {
    const int i = blockIdx.x * BLOCK + threadIdx.x;
    if (i < n) v[i] = i;
}
__global__ __launch_bounds__(BLOCK) void k_perm_keys(int mode, const int* perm, const int* idx, const int* lag,
                                                     const unsigned* keys, int n, unsigned* out) {
    const int i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n) return;
    const int j = perm ? perm[i] : i;
    if (mode == 0) {
        const int s = idx ? idx[j] : j;
        out[i] = (unsigned)(lag ? lag[s] : s);
    } else {
        out[i] = keys[j];
    }
}
__global__ __launch_bounds__(BLOCK) void k_perm_list(const int* perm, const int* idx, const double* xs,
                                                     const int* cells, int ndim, int n, int* idx_out, double* xs_out,
                                                     int* cells_out) {
    const int i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n) return;
    const int j = perm[i];
    idx_out[i] = idx[j];
    if (xs_out)
        for (int k = 0; k < ndim; ++k) xs_out[(int64_t)ndim * i + k] = xs[(int64_t)ndim * j + k];
    if (cells_out)
        for (int k = 0; k < ndim; ++k) cells_out[(int64_t)ndim * i + k] = cells[(int64_t)ndim * j + k];
}
__global__ __launch_bounds__(BLOCK) void k_compact_list(const int* flag, const int* pos, const int* idx,
                                                        const double* xs, const int* cells, int ndim, int n,
                                                        int* idx_out, double* xs_out, int* cells_out) {
    const int i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n || !flag[i]) return;
    const int o = pos[i];
    idx_out[o] = idx[i];
    if (xs_out)
        for (int k = 0; k < ndim; ++k) xs_out[(int64_t)ndim * o + k] = xs[(int64_t)ndim * i + k];
    if (cells_out)
        for (int k = 0; k < ndim; ++k) cells_out[(int64_t)ndim * o + k] = cells[(int64_t)ndim * i + k];
}
__global__ __launch_bounds__(BLOCK) void k_in_box_flags(const int* cells, int ndim, int n, int lo0, int lo1, int lo2,
                                                        int hi0, int hi1, int hi2, int* flag) {
    const int i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n) return;
    const int lo[3] = {lo0, lo1, lo2}, hi[3] = {hi0, hi1, hi2};
    bool in = true;
    for (int k = 0; k < ndim; ++k) {
        const int c = cells[(int64_t)ndim * i + k];
        in = in && c >= lo[k] && c <= hi[k];
    }
    flag[i] = in ? 1 : 0;
}
// computeNodeDistribution (LDataManager.cpp:2874-2947) for one patch: key =
// patch-box linear index (local nodes, numbered first), then ncell + ghost-box
// linear index (the nonlocal nodes in the ghost cells), 0xffffffff outside.
__global__ __launch_bounds__(BLOCK) void k_node_keys(ImageDesc d, const double* X, int n, unsigned* keys) {
    const int i0 = blockIdx.x * BLOCK + threadIdx.x;
    const int i = min(i0, n - 1);  // every lane reaches the wave count below
    int c[3] = {0, 0, 0};
    cell_index(d, X + (int64_t)d.ndim * i, c);
    bool in = true, ing = true;
    unsigned kin = 0, sin = 1, kg = 0, sg = 1;
    for (int k = 0; k < d.ndim; ++k) {
        const int nk = d.ihi[k] - d.ilo[k] + 1;
        in = in && c[k] >= d.ilo[k] && c[k] <= d.ihi[k];
        ing = ing && c[k] >= d.ilo[k] - d.ghost && c[k] <= d.ihi[k] + d.ghost;
        kin += (unsigned)(c[k] - d.ilo[k]) * sin;
        sin *= (unsigned)nk;
        kg += (unsigned)(c[k] - (d.ilo[k] - d.ghost)) * sg;
        sg *= (unsigned)(nk + 2 * d.ghost);
    }
    keys[i] = in ? kin : (ing ? sin + kg : 0xffffffffu);
}
__global__ __launch_bounds__(BLOCK) void k_unique_flags(const unsigned* skeys, const int* sorder, const int* lag, int n,
                                                        int* flag) {
    const int i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n) return;
    bool first = i == 0 || skeys[i] != skeys[i - 1];
    if (!first) {
        const int a = sorder[i], b = sorder[i - 1];
        first = (lag ? lag[a] : a) != (lag ? lag[b] : b);
    }
    flag[i] = first && skeys[i] != 0xffffffffu ? 1 : 0;
}
// counter += the wave's true predicates, one atomic from the wave (per-lane
// atomics on one address serialise); every lane of the wave must call it
__device__ __forceinline__ void wave_count(int* counter, bool pred) {
    const unsigned long long m = __ballot(pred);
    if (m && (threadIdx.x & 63) == 0) atomicAdd(counter, __popcll(m));
}

__global__ __launch_bounds__(BLOCK) void k_compact(const int* sorder, const int* flag, const int* pos,
                                                   const unsigned* skeys, unsigned local_end, unsigned ghost_end, int n,
                                                   int* out, int* counts) {
    const int i = blockIdx.x * BLOCK + threadIdx.x;
    const bool f = i < n && flag[i];
    const bool loc = f && skeys[i] < local_end;
    if (f) out[pos[i]] = sorder[i];
    wave_count(counts, loc);           // one atomic per wave and counter
    wave_count(counts + 1, f && !loc);
}
// *out (zeroed by the caller) += the sum of v[0..n) in 64 bits: the range check of a 32-bit
// scan of per-entry counts, run only where the counts could reach 2^31.  A block's waves
// sum in LDS and one atomic leaves each of at most 256 blocks (per-wave atomics on one
// address serialise: 0.1 ms for 1e7 counts; one a block of 256 threads, 0.27 ms).
__global__ __launch_bounds__(BLOCK) void k_sum64(const int* v, int n, unsigned long long* out) {
    __shared__ unsigned long long ws[BLOCK / 64];
    unsigned long long t = 0;
    for (int i = blockIdx.x * BLOCK + threadIdx.x; i < n; i += gridDim.x * BLOCK) t += (unsigned)v[i];
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) t += __shfl_xor(t, d);
    if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = t;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long b = 0;
        for (int w = 0; w < BLOCK / 64; ++w) b += ws[w];
        if (b) atomicAdd(out, b);
    }
}
hipError_t launch_sum64(const int* v, int n, unsigned long long* out, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_sum64, dim3(std::min((n + BLOCK - 1) / BLOCK, 256)), dim3(BLOCK), 0, s, v, n, out);
    return hipGetLastError();
}
hipError_t launch_iota(int* v, int n, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_iota, dim3((n + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, s, v, n);
    return hipGetLastError();
}
hipError_t launch_perm_keys(int mode, const int* perm, const int* idx, const int* lag, const unsigned* keys, int n,
                            unsigned* out, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_perm_keys, dim3((n + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, s, mode, perm, idx, lag, keys, n,
                       out);
    return hipGetLastError();
}
hipError_t launch_perm_list(const int* perm, const int* idx, const double* xs, const int* cells, int ndim, int n,
                            int* idx_out, double* xs_out, int* cells_out, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_perm_list, dim3((n + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, s, perm, idx, xs, cells, ndim, n,
                       idx_out, xs_out, cells_out);
    return hipGetLastError();
}
hipError_t launch_compact_list(const int* flag, const int* pos, const int* idx, const double* xs, const int* cells,
                               int ndim, int n, int* idx_out, double* xs_out, int* cells_out, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_compact_list, dim3((n + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, s, flag, pos, idx, xs, cells,
                       ndim, n, idx_out, xs_out, cells_out);
    return hipGetLastError();
}
hipError_t launch_in_box_flags(const int* cells, int ndim, int n, const int* lo, const int* hi, int* flag,
                               hipStream_t s) {
    if (n <= 0) return hipSuccess;
    int l[3] = {0, 0, 0}, h[3] = {0, 0, 0};
    for (int k = 0; k < ndim; ++k) {
        l[k] = lo[k];
        h[k] = hi[k];
    }
    hipLaunchKernelGGL(k_in_box_flags, dim3((n + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, s, cells, ndim, n, l[0], l[1],
                       l[2], h[0], h[1], h[2], flag);
    return hipGetLastError();
}
hipError_t launch_node_keys(const ImageDesc& d, const double* X, int n, unsigned* keys, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_node_keys, dim3((n + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, s, d, X, n, keys);
    return hipGetLastError();
}
// ---------------------------------------------------------------------------
// level numbering: LDataManager::computeNodeDistribution (LDataManager.cpp:
// 2874-2947) over the local patches of a level
// ---------------------------------------------------------------------------
__device__ __forceinline__ int floordiv(int a, int b) { return a >= 0 ? a / b : -((-a + b - 1) / b); }
// floor(a / L.n[k]) from a float estimate corrected by one step (exact: |a| < 2^22 keeps the
// estimate within one of the quotient; larger |a| divide): the level kernels' tile searches
// take ~20 of these a marker, each a ~30-instruction integer division otherwise
__device__ __forceinline__ int lfloordiv(const LevelNum& L, int a, int k) {
    const int b = L.n[k];
    if (a >= (1 << 22) || a <= -(1 << 22)) return floordiv(a, b);
    int q = (int)floorf((float)a * L.rn[k]);
    const int r = a - q * b;
    q += r < 0 ? -1 : (r >= b ? 1 : 0);
    return q;
}

__global__ __launch_bounds__(BLOCK) void k_level_node_keys(LevelNum L, const int* tab, const double* X, int n,
                                                           unsigned* lkey, unsigned* ckey) {
    const int s = blockIdx.x * BLOCK + threadIdx.x;
    if (s >= n) return;
    const int nd = L.ndim;
    int c[3] = {0, 0, 0};
    for (int k = 0; k < nd; ++k) {  // IndexUtilities::getCellIndex, IndexUtilities-inl.h:66-89
        const double x = X[(int64_t)nd * s + k];
        const double dl = x - L.xlo[k], du = x - L.xup[k];
        if (fabs(dl) <= fabs(du)) c[k] = L.dom_lo[k] + (int)floor(dl / L.dx[k]);
        else c[k] = L.dom_hi[k] + (int)floor(du / L.dx[k]) + 1;
    }
    const unsigned pcells = (unsigned)L.n[0] * (nd > 1 ? L.n[1] : 1) * (nd > 2 ? L.n[2] : 1);
    unsigned gcells = 1;
    for (int k = 0; k < nd; ++k) gcells *= (unsigned)(L.n[k] + 2 * L.g);
    // the tile (patch) of a cell; -1 outside the table or not local
    auto patch_of = [&](const int* cc, int* t) {
        int lin = 0, str = 1;
        for (int k = 0; k < nd; ++k) {
            t[k] = lfloordiv(L, cc[k] - L.org[k], k);
            if (t[k] < 0 || t[k] >= L.nt[k]) return -1;
            lin += t[k] * str;
            str *= L.nt[k];
        }
        return tab[lin];
    };
    int t[3] = {0, 0, 0};
    const int q = patch_of(c, t);
    if (q >= 0) {  // a local node: its patch's box cells in box order, x fastest
        unsigned k0 = 0, str = 1;
        for (int k = 0; k < nd; ++k) {
            k0 += (unsigned)(c[k] - (L.org[k] + t[k] * L.n[k])) * str;
            str *= (unsigned)L.n[k];
        }
        lkey[s] = (unsigned)q * pcells + k0;
        ckey[s] = 0u;
        return;
    }
    // ghost cells of local patches (periodic images included): the first sighting
    // in patch order, each patch's ghost box in box order
    unsigned best = 0xffffffffu;
    const int nsh = nd == 3 ? 27 : 9;
    for (int j = 0; j < nsh; ++j) {
        const int sh[3] = {j % 3 - 1, (j / 3) % 3 - 1, nd == 3 ? j / 9 - 1 : 0};
        bool ok = true;
        int ci[3] = {0, 0, 0};
        for (int k = 0; k < nd; ++k) {
            if (sh[k] != 0 && !L.periodic[k]) ok = false;
            ci[k] = c[k] + sh[k] * (L.dom_hi[k] - L.dom_lo[k] + 1);
        }
        if (!ok) continue;
        for (int m = 0; m < nsh; ++m) {  // the patches around the image's tile
            const int o[3] = {m % 3 - 1, (m / 3) % 3 - 1, nd == 3 ? m / 9 - 1 : 0};
            int tt[3] = {0, 0, 0}, lin = 0, str = 1;
            bool in = true;
            for (int k = 0; k < nd; ++k) {
                tt[k] = lfloordiv(L, ci[k] - L.org[k], k) + o[k];
                in = in && tt[k] >= 0 && tt[k] < L.nt[k];
                lin += tt[k] * str;
                str *= L.nt[k];
            }
            if (!in) continue;
            const int qq = tab[lin];
            if (qq < 0) continue;
            unsigned gk = 0, gs = 1;
            for (int k = 0; k < nd; ++k) {
                const int lo = L.org[k] + tt[k] * L.n[k] - L.g;
                const int r = ci[k] - lo;
                in = in && r >= 0 && r < L.n[k] + 2 * L.g;
                gk += (unsigned)r * gs;
                gs *= (unsigned)(L.n[k] + 2 * L.g);
            }
            if (!in) continue;
            const unsigned key = (unsigned)qq * gcells + gk;
            best = key < best ? key : best;
        }
    }
    lkey[s] = 0xffffffffu;
    ckey[s] = best == 0xffffffffu ? 0xffffffffu : best + 1u;
}
hipError_t launch_level_node_keys(const LevelNum& L, const int* tab, const double* X, int n, unsigned* lkey,
                                  unsigned* ckey, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_level_node_keys, dim3((n + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, s, L, tab, X, n, lkey, ckey);
    return hipGetLastError();
}
// ---------------------------------------------------------------------------
// a level's index lists in one pass: LIndexSetData::cacheLocalIndices
// (LIndexSetData.cpp:83-169) over every local patch of the level
// ---------------------------------------------------------------------------
// getCellIndex in the domain frame (IndexUtilities-inl.h:66-89), as k_level_node_keys
__device__ __forceinline__ void level_cell(const LevelNum& L, const double* X, int s, int* c) {
    for (int k = 0; k < 3; ++k) c[k] = 0;
    for (int k = 0; k < L.ndim; ++k) {
        const double x = X[(int64_t)L.ndim * s + k];
        const double dl = x - L.xlo[k], du = x - L.xup[k];
        if (fabs(dl) <= fabs(du)) c[k] = L.dom_lo[k] + (int)floor(dl / L.dx[k]);
        else c[k] = L.dom_hi[k] + (int)floor(du / L.dx[k]) + 1;
    }
}
// f(j, q, key) for every periodic image j (shift (j % 3 - 1, j / 3 % 3 - 1, j / 9 - 1) in
// domain extents; non-periodic dims unshifted) of cell c and every local patch q whose ghost
// box holds the image's cell, key = q * (ghost-box cells) + the cell's ghost-box index (x
// fastest); images and patches in increasing (j, tile) order
template <typename F>
__device__ __forceinline__ void level_ghost_visit(const LevelNum& L, const int* tab, const int* c, F&& f) {
    const int nd = L.ndim;
    unsigned gcells = 1;
    for (int k = 0; k < nd; ++k) gcells *= (unsigned)(L.n[k] + 2 * L.g);
    // per dim and shift s - 1 (s = 0, 1, 2): the image's cell and the tiles whose ghost box
    // [org + t n - g, org + t n + n - 1 + g] holds it (empty: no such image here) -- a
    // marker away from the domain's faces has one image, its own
    int ci[3][3], tlo[3][3], thi[3][3];
    for (int k = 0; k < 3; ++k)
        for (int s = 0; s < 3; ++s) {
            ci[k][s] = 0;
            tlo[k][s] = 0;
            thi[k][s] = (k >= nd && s == 1) ? 0 : -1;  // a missing dim: its one unshifted "tile"
        }
    for (int k = 0; k < nd; ++k)
        for (int s = 0; s < 3; ++s) {
            if (s != 1 && !L.periodic[k]) continue;
            const int x = c[k] + (s - 1) * (L.dom_hi[k] - L.dom_lo[k] + 1);
            ci[k][s] = x;
            tlo[k][s] = max(-lfloordiv(L, -(x - L.org[k] - L.n[k] + 1 - L.g), k), 0);
            thi[k][s] = min(lfloordiv(L, x - L.org[k] + L.g, k), L.nt[k] - 1);
        }
    for (int sz = 0; sz < 3; ++sz) {
        if (tlo[2][sz] > thi[2][sz]) continue;
        for (int sy = 0; sy < 3; ++sy) {
            if (tlo[1][sy] > thi[1][sy]) continue;
            for (int sx = 0; sx < 3; ++sx) {
                if (tlo[0][sx] > thi[0][sx]) continue;
                const int j = sx + 3 * sy + 9 * sz;
                const int sv[3] = {sx, sy, sz};
                for (int tz = tlo[2][sz]; tz <= thi[2][sz]; ++tz)
                    for (int ty = tlo[1][sy]; ty <= thi[1][sy]; ++ty)
                        for (int tx = tlo[0][sx]; tx <= thi[0][sx]; ++tx) {
                            const int tt[3] = {tx, ty, tz};
                            int lin = 0, str = 1;
                            for (int k = 0; k < nd; ++k) {
                                lin += tt[k] * str;
                                str *= L.nt[k];
                            }
                            const int q = tab[lin];
                            if (q < 0) continue;
                            unsigned gk = 0, gs = 1;
                            for (int k = 0; k < nd; ++k) {
                                gk += (unsigned)(ci[k][sv[k]] - (L.org[k] + tt[k] * L.n[k] - L.g)) * gs;
                                gs *= (unsigned)(L.n[k] + 2 * L.g);
                            }
                            f(j, q, (unsigned)q * gcells + gk);
                        }
            }
        }
    }
}
// per marker: its interior key (patch q * patch cells + the cell's box index; 0xffffffff
// in no local patch box) and its number of ghost-box entries.  bypatch: the keys are the
// patch alone (npatch: none) -- the lists in marker order within a patch
// a marker's interior key (ikey[s]) and its count of ghost-box entries
__device__ __forceinline__ int level_list_key(LevelNum L, const int* tab, const double* X, int s, unsigned* ikey,
                                                   int bypatch, int npatch) {
    const int nd = L.ndim;
    int c[3];
    level_cell(L, X, s, c);
    unsigned key = 0xffffffffu, pcells = 1, k0 = 0;
    int lin = 0, str = 1, t[3] = {0, 0, 0};
    bool in = true;
    for (int k = 0; k < nd; ++k) {
        t[k] = lfloordiv(L, c[k] - L.org[k], k);
        in = in && t[k] >= 0 && t[k] < L.nt[k];
        lin += t[k] * str;
        str *= L.nt[k];
        k0 += (unsigned)(c[k] - (L.org[k] + t[k] * L.n[k])) * pcells;
        pcells *= (unsigned)L.n[k];
    }
    if (in && tab[lin] >= 0) key = bypatch ? (unsigned)tab[lin] : (unsigned)tab[lin] * pcells + k0;
    else if (bypatch) key = (unsigned)npatch;
    ikey[s] = key;
    int cnt = 0;
    level_ghost_visit(L, tab, c, [&](int, int, unsigned) { ++cnt; });
    return cnt;
}
__global__ __launch_bounds__(BLOCK) void k_level_list_keys(LevelNum L, const int* tab, const double* X, int n,
                                                           unsigned* ikey, int* gcnt, int bypatch, int npatch) {
    const int s = blockIdx.x * BLOCK + threadIdx.x;
    if (s < n) gcnt[s] = level_list_key(L, tab, X, s, ikey, bypatch, npatch);
}
// the ghost-box entries at goff[s]: key, entry id (the stable sort's value), marker, image
__global__ __launch_bounds__(BLOCK) void k_level_list_write(LevelNum L, const int* tab, const double* X, int n,
                                                            const int* goff, unsigned* gkey, int* gid, int* gsrc,
                                                            int* gimg, int bypatch) {
    const int s = blockIdx.x * BLOCK + threadIdx.x;
    if (s >= n) return;
    int c[3];
    level_cell(L, X, s, c);
    int o = goff[s];
    level_ghost_visit(L, tab, c, [&](int j, int q, unsigned key) {
        gkey[o] = bypatch ? (unsigned)q : key;
        gid[o] = o;
        gsrc[o] = s;
        gimg[o] = j;
        ++o;
    });
}
// the sorted entries out: marker index and its periodic shift (sh * domain length per dim)
__global__ __launch_bounds__(BLOCK) void k_level_list_out(LevelNum L, const int* sid, const int* gsrc,
                                                          const int* gimg, int total, int* idx, double* xs) {
    const int i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= total) return;
    const int e = sid[i];
    idx[i] = gsrc[e];
    if (xs) {
        const int j = gimg[e];
        const int sh[3] = {j % 3 - 1, (j / 3) % 3 - 1, j / 9 - 1};
        for (int k = 0; k < L.ndim; ++k)
            xs[(int64_t)L.ndim * i + k] = (double)sh[k] * ((double)(L.dom_hi[k] - L.dom_lo[k] + 1) * L.dx[k]);
    }
}
// off[q] = the first sorted key >= q * per (q = 0 .. npatch; keys of no patch sort last)
__global__ __launch_bounds__(BLOCK) void k_key_offsets(const unsigned* skeys, int n, unsigned per, int npatch,
                                                       int* off) {
    const int q = blockIdx.x * BLOCK + threadIdx.x;
    if (q > npatch) return;
    const unsigned long long b = (unsigned long long)q * per;
    int lo = 0, hi = n;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if ((unsigned long long)skeys[mid] < b) lo = mid + 1;
        else hi = mid;
    }
    off[q] = lo;
}
hipError_t launch_level_list_keys(const LevelNum& L, const int* tab, const double* X, int n, unsigned* ikey,
                                  int* gcnt, int bypatch, int npatch, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_level_list_keys, dim3((n + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, s, L, tab, X, n, ikey, gcnt,
                       bypatch, npatch);
    return hipGetLastError();
}
hipError_t launch_level_list_write(const LevelNum& L, const int* tab, const double* X, int n, const int* goff,
                                   unsigned* gkey, int* gid, int* gsrc, int* gimg, int bypatch, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_level_list_write, dim3((n + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, s, L, tab, X, n, goff, gkey,
                       gid, gsrc, gimg, bypatch);
    return hipGetLastError();
}
hipError_t launch_level_list_out(const LevelNum& L, const int* sid, const int* gsrc, const int* gimg, int total,
                                 int* idx, double* xs, hipStream_t s) {
    if (total <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_level_list_out, dim3((total + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, s, L, sid, gsrc, gimg,
                       total, idx, xs);
    return hipGetLastError();
}
hipError_t launch_key_offsets(const unsigned* skeys, int n, unsigned per, int npatch, int* off, hipStream_t s) {
    hipLaunchKernelGGL(k_key_offsets, dim3((npatch + 1 + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, s, skeys, n, per, npatch,
                       off);
    return hipGetLastError();
}
// entry i of the list sorted by (lag, ckey): the first of its lag run, and that run
// has no local node (ckey 0 sorts first) -- a nonlocal node at its first sighting
__global__ __launch_bounds__(BLOCK) void k_nonlocal_flags(const unsigned* sckey, const int* sorder, const int* lag,
                                                          int n, int* flag) {
    const int i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n) return;
    const int a = sorder[i];
    const bool first = i == 0 || (lag ? lag[sorder[i - 1]] : sorder[i - 1]) != (lag ? lag[a] : a);
    flag[i] = first && sckey[i] != 0u && sckey[i] != 0xffffffffu ? 1 : 0;
}
hipError_t launch_nonlocal_flags(const unsigned* sckey, const int* sorder, const int* lag, int n, int* flag,
                                 hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_nonlocal_flags, dim3((n + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, s, sckey, sorder, lag, n, flag);
    return hipGetLastError();
}
__global__ __launch_bounds__(BLOCK) void k_take_keys(const unsigned* keys, const int* idx, int n, unsigned* out) {
    const int i = blockIdx.x * BLOCK + threadIdx.x;
    if (i < n) out[i] = keys[idx[i]];
}
hipError_t launch_take_keys(const unsigned* keys, const int* idx, int n, unsigned* out, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_take_keys, dim3((n + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, s, keys, idx, n, out);
    return hipGetLastError();
}
// endDataRedistribution's VecScatter of an LData (LDataManager.cpp:1823-1917): the
// new node i takes the old row order[i]; 3-deep rows as one 24-byte record
__global__ __launch_bounds__(BLOCK) void k_rows_gather(const int* order, int n, const double* in, int depth,
                                                       double* out) {
    const int i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n) return;
    const int64_t j = order[i];
    if (depth == 3) {
        struct R3 {
            double v[3];
        };
        *reinterpret_cast<R3*>(out + 3 * (int64_t)i) = *reinterpret_cast<const R3*>(in + 3 * j);
    } else {
        for (int k = 0; k < depth; ++k) out[(int64_t)depth * i + k] = in[(int64_t)depth * j + k];
    }
}
hipError_t launch_rows_gather(const int* order, int n, const double* in, int depth, double* out, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_rows_gather, dim3((n + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, s, order, n, in, depth, out);
    return hipGetLastError();
}

hipError_t launch_unique_flags(const unsigned* skeys, const int* sorder, const int* lag, int n, int* flag,
                               hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_unique_flags, dim3((n + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, s, skeys, sorder, lag, n, flag);
    return hipGetLastError();
}
hipError_t launch_compact(const int* sorder, const int* flag, const int* pos, const unsigned* skeys,
                          unsigned local_end, unsigned ghost_end, int n, int* out, int* counts, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    (void)ghost_end;
    hipLaunchKernelGGL(k_compact, dim3((n + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, s, sorder, flag, pos, skeys,
                       local_end, ghost_end, n, out, counts);
    return hipGetLastError();
}

// Local numbering keys (LDataManager::computeNodeDistribution, LDataManager.cpp:
// 2839-3027): the linear index of the marker's cell in the patch box, x fastest
// (the box iteration order of LNodeSetData), by getCellIndex; markers whose
// cell is outside the box get key ncells (numbered last).  vals = input index,
// so a stable sort keeps input order within a cell.
__global__ __launch_bounds__(BLOCK) void k_cell_keys(ImageDesc d, const double* X, int n, unsigned ncells,
                                                     unsigned* keys, int* vals, int* inside) {
    const int i0 = blockIdx.x * BLOCK + threadIdx.x;
    const int i = min(i0, n - 1);  // every lane reaches the wave count below
    int c[3] = {0, 0, 0};
    cell_index(d, X + (int64_t)d.ndim * i, c);
    unsigned key = 0, stride = 1;
    bool in = true;
    for (int k = 0; k < d.ndim; ++k) {
        in = in && c[k] >= d.ilo[k] && c[k] <= d.ihi[k];
        key += (unsigned)(c[k] - d.ilo[k]) * stride;
        stride *= (unsigned)(d.ihi[k] - d.ilo[k] + 1);
    }
    if (i0 < n) {
        keys[i] = in ? key : ncells;
        vals[i] = i;
    }
    wave_count(inside, in && i0 < n);
}

hipError_t launch_cell_keys(const ImageDesc& d, const double* X, int n, unsigned ncells, unsigned* keys, int* vals,
                            int* inside, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_cell_keys, dim3((n + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, s, d, X, n, ncells, keys, vals,
                       inside);
    return hipGetLastError();
}

hipError_t launch_image_count(const ImageDesc& d, const double* X, int n, int* counts, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_image_count, dim3((n + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, s, d, X, n, counts);
    return hipGetLastError();
}
hipError_t launch_image_write(const ImageDesc& d, const double* X, int n, const int* offsets, int* idx,
                              double* xshift, unsigned* cellkey, int* cells, int capacity, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_image_write, dim3((n + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, s, d, X, n, offsets, idx,
                       xshift, cellkey, cells, capacity);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// interpolation lists that name a marker more than once (the ghost-box list of
// LIndexSetData holds a marker and its periodic images): the Fortran l-loop
// overwrites V(:,s) entry after entry, so the LAST list entry of s wins
// (lagrangian_interaction3d.f.m4:1366-1382).  qdst[e] = s for that entry, -1
// for the earlier ones (their sums go to the sink).
// ---------------------------------------------------------------------------
// grid-stride max, reduced in the block: one atomic per block (one per wave on
// a single address serialised 10M entries into 1.8 ms)
__global__ __launch_bounds__(BLOCK) void k_max_index(const int* idx, int n, int* out) {
    __shared__ int wmax[BLOCK / 64];
    int v = -1;
    for (long l = (long)blockIdx.x * BLOCK + threadIdx.x; l < n; l += (long)gridDim.x * BLOCK) v = max(v, idx[l]);
    for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o));
    if ((threadIdx.x & 63) == 0) wmax[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < BLOCK / 64; ++w) v = max(v, wmax[w]);
        if (v >= 0) atomicMax(out, v);
    }
}
__global__ __launch_bounds__(BLOCK) void k_last_entry(const int* idx, int n, int* last) {
    const int l = blockIdx.x * BLOCK + threadIdx.x;
    if (l < n) atomicMax(last + idx[l], l);
}
__global__ __launch_bounds__(BLOCK) void k_qdst(const int* sorted_l, const int* sorted_s, const int* last, int n,
                                                int* qdst, int* ndup) {
    const int e = blockIdx.x * BLOCK + threadIdx.x;
    if (e >= n) return;
    const int s = sorted_s[e];
    const bool keep = last[s] == sorted_l[e];
    qdst[e] = keep ? s : -1;
    if (!keep) atomicAdd(ndup, 1);
}
hipError_t launch_max_index(const int* idx, int n, int* out, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_max_index, dim3(std::min((n + BLOCK - 1) / BLOCK, 2048)), dim3(BLOCK), 0, s, idx, n, out);
    return hipGetLastError();
}
hipError_t launch_dedup(const int* indices, const int* sorted_l, const int* sorted_s, int n, int* last, int* qdst,
                        int* ndup, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    const dim3 g((n + BLOCK - 1) / BLOCK);
    hipLaunchKernelGGL(k_last_entry, g, dim3(BLOCK), 0, s, indices, n, last);
    hipLaunchKernelGGL(k_qdst, g, dim3(BLOCK), 0, s, sorted_l, sorted_s, last, n, qdst, ndup);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// marker position update (IBMethod::eulerStep / midpointStep / trapezoidalStep,
// IBMethod.cpp:619-681): PETSc VecWAXPY w = alpha x + y and VecAXPY y += alpha x,
// each a rounded multiply then a rounded add (built with -ffp-contract=off, so
// no fma), elementwise over the n doubles of the (M, NDIM) arrays.  HBM-bound:
// 16-byte accesses, pairs of doubles per lane when every array is 16-byte aligned,
// PU_UNROLL items a lane with every load issued before the first store (X may be Xn:
// each element is read and written by one lane, read first).  Round 6: 1.57 ms for
// cfg4's 1e8 markers (7.2 GB, 4.6 TB/s) with one item a lane in a grid-stride loop.
// ---------------------------------------------------------------------------
constexpr int PU_UNROLL = 4;
template <bool TRAP, typename V>
__device__ __forceinline__ V pu_step(double dt, const V& x, const V& u, const V& v) {
    if constexpr (sizeof(V) == 16) {
        V w;
        if constexpr (TRAP) {
            const double h = 0.5 * dt;
            w.x = (h * u.x + x.x) + h * v.x;
            w.y = (h * u.y + x.y) + h * v.y;
        } else {
            w.x = dt * u.x + x.x;
            w.y = dt * u.y + x.y;
        }
        return w;
    } else {
        if constexpr (TRAP) {
            const double h = 0.5 * dt;
            return (h * u + x) + h * v;
        } else {
            return dt * u + x;
        }
    }
}
template <bool TRAP, typename V>
__global__ __launch_bounds__(BLOCK) void k_position_update(long n, double dt, const V* X, const V* U0, const V* U1,
                                                           V* Xn) {
    const long i0 = (long)blockIdx.x * (BLOCK * PU_UNROLL) + threadIdx.x;
    V x[PU_UNROLL], u[PU_UNROLL], v[PU_UNROLL];
#pragma unroll
    for (int k = 0; k < PU_UNROLL; ++k) {
        const long i = i0 + (long)k * BLOCK;
        if (i < n) {
            x[k] = X[i];
            u[k] = U0[i];
            if constexpr (TRAP) v[k] = U1[i];
            else v[k] = u[k];
        }
    }
#pragma unroll
    for (int k = 0; k < PU_UNROLL; ++k) {
        const long i = i0 + (long)k * BLOCK;
        if (i < n) Xn[i] = pu_step<TRAP, V>(dt, x[k], u[k], v[k]);
    }
}

hipError_t launch_position_update(int scheme, long n, double dt, const double* X, const double* U0, const double* U1,
                                  double* Xn, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    const bool trap = scheme == 2;
    auto al = [](const void* q) { return q == nullptr || ((uintptr_t)q & 15u) == 0; };
    const bool vec = (n % 2 == 0) && al(X) && al(U0) && al(U1) && al(Xn);
    const long items = vec ? n / 2 : n;
    const long grid = (items + BLOCK * PU_UNROLL - 1) / (BLOCK * PU_UNROLL);
    if (grid > 0x7fffffffL) return hipErrorInvalidValue;
    if (vec) {
        using V = double2;
        auto x = (const V*)X;
        auto u0 = (const V*)U0;
        auto u1 = (const V*)U1;
        auto xn = (V*)Xn;
        if (trap) hipLaunchKernelGGL((k_position_update<true, V>), dim3((unsigned)grid), dim3(BLOCK), 0, s, items, dt, x, u0, u1, xn);
        else hipLaunchKernelGGL((k_position_update<false, V>), dim3((unsigned)grid), dim3(BLOCK), 0, s, items, dt, x, u0, u1, xn);
    } else {
        if (trap) hipLaunchKernelGGL((k_position_update<true, double>), dim3((unsigned)grid), dim3(BLOCK), 0, s, items, dt, X, U0, U1, Xn);
        else hipLaunchKernelGGL((k_position_update<false, double>), dim3((unsigned)grid), dim3(BLOCK), 0, s, items, dt, X, U0, U1, Xn);
    }
    return hipGetLastError();
}

}  // namespace ibtk_le

namespace ibtk_le {

// ---------------------------------------------------------------------------
// z-slab marker migration fused with the position update (the per-step
// redistribution SURVEY.md 8(e) asks for; the reference's LDataManager.cpp:
// 1504-1959 at regrid).  Pass 1 (k_slab_update): X_new = the update of
// ibtk_le_position_update (same rounding), wrapped into [0, L) per dim exactly as
// torch.remainder does it (fmod, then + L if negative, then - L if it reached L),
// the owner of the wrapped z cell (IndexUtilities::getCellIndex, clamped), and
// the class: 0 stays, 1 to the lower neighbour, 2 to the upper, 3 further; the
// class counts per block.  Pass 2 (k_slab_partition), after an exclusive scan of
// the class-major block counts: a stable partition of the marker indices,
// [stay | down | up | far], each in input order.  Deterministic, no host sync.
// ---------------------------------------------------------------------------
__device__ __forceinline__ double wrap_like_torch(double x, double L) {
    double r = fmod(x, L);
    if (r != 0.0 && r < 0.0) r = r + L;
    if (r >= L) r = r - L;
    return r;
}

template <int SCHEME>
__global__ __launch_bounds__(BLOCK) void k_slab_update(long M, double dt, const double* X, const double* U0,
                                                       const double* U1, double* Xn, SlabMig g, unsigned char* cls,
                                                       int* bcount, int nb) {
    __shared__ int cnt[4];
    if (threadIdx.x < 4) cnt[threadIdx.x] = 0;
    __syncthreads();
    const long i = (long)blockIdx.x * BLOCK + threadIdx.x;
    const long Mv = g.n_dev ? min((long)*g.n_dev, M) : M;
    int c = -1;
    if (i < M && i >= Mv) cls[i] = 255;  // unused row of a fixed-capacity list
    if (i < Mv) {
        double w[3];
#pragma unroll
        for (int d = 0; d < 3; ++d) {
            const long k = 3 * i + d;
            double x;
            if constexpr (SCHEME == 2) {
                const double h = 0.5 * dt;
                x = (h * U0[k] + X[k]) + h * U1[k];
            } else {
                x = dt * U0[k] + X[k];
            }
            w[d] = wrap_like_torch(x, g.L[d]);
            Xn[k] = w[d];
        }
        const long cz = min(max((long)floor(w[2] / g.dz), 0L), (long)g.Nz - 1);
        const int owner = (int)(cz / g.nz);
        const int down = (g.rank - 1 + g.P) % g.P, up = (g.rank + 1) % g.P;
        c = owner == g.rank ? 0 : (owner == down ? 1 : (owner == up ? 2 : 3));
        cls[i] = (unsigned char)c;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const unsigned long long b = __ballot(c == k);
        if ((threadIdx.x & 63) == 0 && b) atomicAdd(&cnt[k], __popcll(b));
    }
    __syncthreads();
    if (threadIdx.x < 4) bcount[threadIdx.x * nb + blockIdx.x] = cnt[threadIdx.x];
}

__global__ __launch_bounds__(BLOCK) void k_slab_partition(long M, const unsigned char* cls, const int* bcount,
                                                          const int* boff, int nb, int* order, int* counts) {
    __shared__ int wcnt[BLOCK / 64][4];
    const long i = (long)blockIdx.x * BLOCK + threadIdx.x;
    const int c = i < M && cls[i] < 4 ? (int)cls[i] : -1;
    const int w = threadIdx.x >> 6;
    int rank = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const unsigned long long b = __ballot(c == k);
        if (c == k) rank = (int)__builtin_amdgcn_mbcnt_hi((unsigned)(b >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)b, 0u));
        if ((threadIdx.x & 63) == 0) wcnt[w][k] = __popcll(b);
    }
    __syncthreads();
    if (c >= 0) {
        int before = 0;
        for (int v = 0; v < w; ++v) before += wcnt[v][c];
        order[boff[c * nb + blockIdx.x] + before + rank] = (int)i;
    }
    if (blockIdx.x == nb - 1 && threadIdx.x < 4) {
        const int k = threadIdx.x;
        counts[k] = boff[k * nb + nb - 1] + bcount[k * nb + nb - 1] - boff[k * nb];
    }
}

hipError_t launch_slab_update_partition(int scheme, long M, double dt, const double* X, const double* U0,
                                        const double* U1, double* Xn, const SlabMig& g, unsigned char* cls,
                                        int* bcount, int* boff, void* temp, size_t& temp_bytes, int* order,
                                        int* counts, hipStream_t s) {
    const int nb = (int)((M + BLOCK - 1) / BLOCK);
    if (!temp) return launch_scan(nullptr, temp_bytes, bcount, boff, 4 * nb, s);  // size query
    if (scheme == 2)
        hipLaunchKernelGGL(k_slab_update<2>, dim3(nb), dim3(BLOCK), 0, s, M, dt, X, U0, U1, Xn, g, cls, bcount, nb);
    else
        hipLaunchKernelGGL(k_slab_update<0>, dim3(nb), dim3(BLOCK), 0, s, M, dt, X, U0, U1, Xn, g, cls, bcount, nb);
    hipError_t e = launch_scan(temp, temp_bytes, bcount, boff, 4 * nb, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_slab_partition, dim3(nb), dim3(BLOCK), 0, s, M, cls, bcount, boff, nb, order, counts);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// a level's interp on its interior lists, from the binned ghost-box lists
// ---------------------------------------------------------------------------
// the patch of entry l (off: npatch + 1 offsets); the wave's first entry's patch
// is searched once (scalar loads) and kept for the lanes in it (a wave's entries are
// mostly of one patch)
__device__ __forceinline__ int patch_of_entry(const int* off, int npatch, int l) {
    auto search = [&](int v) {
        int lo = 0, hi = npatch - 1;
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (off[mid] <= v) lo = mid;
            else hi = mid - 1;
        }
        return lo;
    };
    const int q = search(__builtin_amdgcn_readfirstlane(l));
    return (off[q] <= l && l < off[q + 1]) ? q : search(l);
}
// gs (ibtk_le_level_select_interior's cache): {the binning's order generation, the one the
// selection was made at}; equal: the selection stands and these kernels return at once
__device__ __forceinline__ bool sel_current(const int* gs) { return gs && gs[0] == gs[1]; }
__global__ __launch_bounds__(BLOCK) void k_interior_owner(const int* int_off, int npatch, const int* int_idx, int n_int,
                                                          int n_markers, int* owner, int* err, const int* gs) {
    if (sel_current(gs)) return;
    const int j = blockIdx.x * BLOCK + threadIdx.x;
    if (j >= n_int) return;
    const int s = int_idx[j];
    if (s < 0 || s >= n_markers) {  // an interior list naming a marker past n_markers
        atomicOr(err, 4);
        return;
    }
    atomicMax(owner + s, patch_of_entry(int_off, npatch, j));
}
hipError_t launch_interior_owner(const int* int_off, int npatch, const int* int_idx, int n_int, int n_markers,
                                 int* owner, int* err, const int* gs, hipStream_t s) {
    if (n_int <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_interior_owner, dim3((n_int + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, s, int_off, npatch, int_idx,
                       n_int, n_markers, owner, err, gs);
    return hipGetLastError();
}
__global__ __launch_bounds__(BLOCK) void k_interior_targets(const int* sorted_l, const int* sorted_s,
                                                            const int* entry_off, int npatch, const double* xshift,
                                                            const int* owner, int n_markers, int n, int* qin,
                                                            int* found, int* err, const int* gs) {
    if (sel_current(gs)) return;  // (uniform over the block: before its barriers)
    const int e = blockIdx.x * BLOCK + threadIdx.x;
    bool keep = false;
    int s = -1;
    if (e < n) {
        const int l = sorted_l[e];
        s = sorted_s[e];
        const bool inr = s >= 0 && s < n_markers;  // a binned list naming a marker past n_markers
        if (!inr) atomicOr(err, 4);
        keep = inr && owner[s] == patch_of_entry(entry_off, npatch, l);
        if (xshift) keep = keep && xshift[3 * (int64_t)l] == 0.0 && xshift[3 * (int64_t)l + 1] == 0.0 &&
                           xshift[3 * (int64_t)l + 2] == 0.0;
        qin[e] = keep ? s : -1;
    }
    // the block's count into one of CHECK_STRIPES counters (one atomic per wave
    // into LDS, one per block into global memory, spread over the stripes: a single
    // global address took 2.1 ms of contention on cfg5's 1.3e7 entries)
    __shared__ int cnt;
    if (threadIdx.x == 0) cnt = 0;
    __syncthreads();
    const unsigned long long b = __ballot(keep);
    if ((threadIdx.x & 63) == 0 && b) atomicAdd(&cnt, __popcll(b));
    __syncthreads();
    if (threadIdx.x == 0 && cnt) atomicAdd(found + (blockIdx.x % CHECK_STRIPES), cnt);
}
hipError_t launch_interior_targets(const int* sorted_l, const int* sorted_s, const int* entry_off, int npatch,
                                   const double* xshift, const int* owner, int n_markers, int n, int* qin, int* found,
                                   int* err, const int* gs, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_interior_targets, dim3((n + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, s, sorted_l, sorted_s,
                       entry_off, npatch, xshift, owner, n_markers, n, qin, found, err, gs);
    return hipGetLastError();
}
// the selection is of the current order: gs[1] = gs[0]
__global__ void k_sel_mark(int* gs) { gs[1] = gs[0]; }
hipError_t launch_sel_mark(int* gs, hipStream_t s) {
    hipLaunchKernelGGL(k_sel_mark, dim3(1), dim3(1), 0, s, gs);
    return hipGetLastError();
}
// fixed-capacity migration: pack the leavers, unpack stayers + arrivals (no host sync)
__global__ __launch_bounds__(BLOCK) void k_mig_pack(const double* rows, int D, const int* order, const int* counts,
                                                    int send_cap, double* send_down, double* send_up, int* err) {
    const int n_stay = counts[0], n_down = counts[1], n_up = counts[2];
    const long t = (long)blockIdx.x * BLOCK + threadIdx.x;
    if (t == 0 && (n_down > send_cap || n_up > send_cap || counts[3] > 0)) atomicOr(err, 8);
    const long tot = (long)send_cap * D;
    if (t >= 2 * tot) return;
    const bool up = t >= tot;
    const long u = up ? t - tot : t;
    const int j = (int)(u / D), d = (int)(u - (long)j * D);
    const int n = up ? n_up : n_down;
    if (j >= n) return;
    const int src = order[n_stay + (up ? n_down : 0) + j];
    (up ? send_up : send_down)[u] = rows[(long)src * D + d];
}
hipError_t launch_mig_pack(const double* rows, int D, const int* order, const int* counts, int send_cap,
                           double* send_down, double* send_up, int* err, hipStream_t s) {
    const long tot = 2L * send_cap * D;
    hipLaunchKernelGGL(k_mig_pack, dim3((unsigned)((tot + BLOCK - 1) / BLOCK + (tot == 0))), dim3(BLOCK), 0, s, rows,
                       D, order, counts, send_cap, send_down, send_up, err);
    return hipGetLastError();
}
__global__ __launch_bounds__(BLOCK) void k_mig_unpack(const double* rows, int D, const int* order, const int* counts,
                                                      const int* rc, const double* from_down, const double* from_up,
                                                      int send_cap, double* out, int out_cap, int* n_out, int* err) {
    const int n_stay = counts[0];
    const int rd = min(rc[0], send_cap), ru = min(rc[1], send_cap);
    const long total = (long)n_stay + rd + ru;
    const long t = (long)blockIdx.x * BLOCK + threadIdx.x;
    if (t == 0) {
        if (rc[0] > send_cap || rc[1] > send_cap || total > out_cap) atomicOr(err, 8);
        *n_out = (int)min(total, (long)out_cap);
    }
    const long i = t / D;
    const int d = (int)(t - i * D);
    if (i >= min(total, (long)out_cap)) return;
    double v;
    if (i < n_stay) v = rows[(long)order[i] * D + d];
    else if (i < n_stay + rd) v = from_down[(i - n_stay) * D + d];
    else v = from_up[(i - n_stay - rd) * D + d];
    out[t] = v;
}
hipError_t launch_mig_unpack(const double* rows, int D, const int* order, const int* counts, const int* rc,
                             const double* from_down, const double* from_up, int send_cap, double* out, int out_cap,
                             int* n_out, int* err, hipStream_t s) {
    const long tot = (long)out_cap * D;
    hipLaunchKernelGGL(k_mig_unpack, dim3((unsigned)((tot + BLOCK - 1) / BLOCK + (tot == 0))), dim3(BLOCK), 0, s, rows,
                       D, order, counts, rc, from_down, from_up, send_cap, out, out_cap, n_out, err);
    return hipGetLastError();
}

__global__ __launch_bounds__(BLOCK) void k_wrap_positions(WrapBox w, long long n, double* X) {
    const long long t = (long long)blockIdx.x * BLOCK + threadIdx.x;
    if (t >= n * w.ndim) return;
    const int d = (int)(t % w.ndim);
    double x = X[t];
    if (w.per[d]) {
        const double L = w.hi[d] - w.lo[d];
        while (x < w.lo[d]) x += L;
        while (x >= w.hi[d]) x -= L;
    }
    // std::max / std::min as LDataManager.cpp:1398-1399 call them ((a < b) ? b : a and
    // (b < a) ? b : a): a NaN coordinate stays NaN (fmax / fmin would clamp it)
    const double lo = w.lo[d], hi = w.hi[d] - 2.220446049250313e-16;  // std::numeric_limits<double>::epsilon()
    x = (x < lo) ? lo : x;
    x = (hi < x) ? hi : x;
    X[t] = x;
}
hipError_t launch_wrap_positions(const WrapBox& w, long long n, double* X, hipStream_t s) {
    const long long tot = n * w.ndim;
    hipLaunchKernelGGL(k_wrap_positions, dim3((unsigned)((tot + BLOCK - 1) / BLOCK)), dim3(BLOCK), 0, s, w, n, X);
    return hipGetLastError();
}

__global__ __launch_bounds__(BLOCK) void k_check_count(const int* count, int ncount, int expect, int* err, int bit,
                                                       const int* gs) {
    if (sel_current(gs)) return;
    __shared__ long long tot;
    if (threadIdx.x == 0) tot = 0;
    __syncthreads();
    long long mine = 0;
    for (int i = threadIdx.x; i < ncount; i += BLOCK) mine += count[i];
    atomicAdd((unsigned long long*)&tot, (unsigned long long)mine);
    __syncthreads();
    if (threadIdx.x == 0 && tot != expect) atomicOr(err, bit);
}
hipError_t launch_check_count(const int* count, int ncount, int expect, int* err, int bit, hipStream_t s,
                              const int* gs) {
    hipLaunchKernelGGL(k_check_count, dim3(1), dim3(BLOCK), 0, s, count, ncount, expect, err, bit, gs);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// USER_DEFINED kernel function (LEInteractor.cpp:3141-3393; host-evaluated weights)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(BLOCK) void k_user_gather(const double* X, const int* indices, const double* Xshift, int n,
                                                       int ndim, double* Xraw, double* Xsh, int* sidx) {
    const int l = blockIdx.x * BLOCK + threadIdx.x;
    if (l >= n) return;
    const int s = indices ? indices[l] : l;
    sidx[l] = s;
    for (int d = 0; d < ndim; ++d) {
        const double x = X[(int64_t)ndim * s + d];
        Xraw[(int64_t)ndim * l + d] = x;
        Xsh[(int64_t)ndim * l + d] = x + (Xshift ? Xshift[(int64_t)ndim * l + d] : 0.0);  // X + X_shift (:3177)
    }
}
hipError_t launch_user_gather(const double* X, const int* indices, const double* Xshift, int n, int ndim, double* Xraw,
                              double* Xsh, int* sidx, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_user_gather, dim3((n + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, s, X, indices, Xshift, n, ndim, Xraw,
                       Xsh, sidx);
    return hipGetLastError();
}

__device__ __forceinline__ int64_t user_off(const CompDesc& cd, int i0, int i1, int i2) {
    return (int64_t)(i0 - cd.lo[0]) + (int64_t)(i1 - cd.lo[1]) * cd.s1 + (int64_t)(i2 - cd.lo[2]) * cd.s2;
}

// Q(d, s) = sum over ic2, ic1, ic0 of w0 w1 w2 q, from 0 (LEInteractor.cpp:3241-3263); the
// last entry naming s writes it, as the sequential l-loop leaves it
__global__ __launch_bounds__(BLOCK) void k_user_interp(UserDesc u) {
    const int l = blockIdx.x * BLOCK + threadIdx.x;
    if (l >= u.n || !u.last[l]) return;
    const int S = u.S;
    const int* lo = u.lo + 3 * l;
    const int* cn = u.cnt + 3 * l;
    const double* w = u.w + (int64_t)3 * S * l;
    double acc = 0.0;
    if (u.ndim == 3) {
        for (int i2 = 0; i2 < cn[2]; ++i2)
            for (int i1 = 0; i1 < cn[1]; ++i1)
                for (int i0 = 0; i0 < cn[0]; ++i0)
                    acc = acc + w[i0] * w[S + i1] * w[2 * S + i2] * u.cd.u[user_off(u.cd, lo[0] + i0, lo[1] + i1, lo[2] + i2)];
    } else {
        for (int i1 = 0; i1 < cn[1]; ++i1)
            for (int i0 = 0; i0 < cn[0]; ++i0)
                acc = acc + w[i0] * w[S + i1] * u.cd.u[user_off(u.cd, lo[0] + i0, lo[1] + i1, u.cd.lo[2])];
    }
    u.Qout[(int64_t)u.Q_depth * u.sidx[l] + u.cd.qcomp] = acc;
}
hipError_t launch_user_interp(const UserDesc& u, hipStream_t s) {
    if (u.n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_user_interp, dim3((u.n + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, s, u);
    return hipGetLastError();
}

// contribution k of entry l (stencil point k, x fastest): w0 w1 [w2] Q(d, s) / (dx0 dx1 [dx2])
// (LEInteractor.cpp:3378-3383), keyed by its array offset; points past the clipped
// stencil are keyed 0xffffffff (sorted last, never summed)
__global__ __launch_bounds__(BLOCK) void k_user_contrib(UserDesc u, unsigned* keys, int* vals, double* contrib) {
    const int S = u.S;
    const int per = u.ndim == 3 ? S * S * S : S * S;
    const int64_t t = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (t >= (int64_t)u.n * per) return;
    const int l = (int)(t / per), k = (int)(t - (int64_t)l * per);
    const int i0 = k % S, i1 = (k / S) % S, i2 = k / (S * S);
    const int* lo = u.lo + 3 * l;
    const int* cn = u.cnt + 3 * l;
    vals[t] = (int)t;
    if (i0 >= cn[0] || i1 >= cn[1] || (u.ndim == 3 && i2 >= cn[2])) {
        keys[t] = 0xffffffffu;
        return;
    }
    const double* w = u.w + (int64_t)3 * S * l;
    const double V = u.Q[(int64_t)u.Q_depth * u.sidx[l] + u.cd.qcomp];
    const double term = u.ndim == 3 ? w[i0] * w[S + i1] * w[2 * S + i2] * V : w[i0] * w[S + i1] * V;
    contrib[t] = term / u.dxprod;
    keys[t] = (unsigned)user_off(u.cd, lo[0] + i0, lo[1] + i1, u.ndim == 3 ? lo[2] + i2 : u.cd.lo[2]);
}
hipError_t launch_user_contrib(const UserDesc& u, unsigned* keys, int* vals, double* contrib, hipStream_t s) {
    const int per = u.ndim == 3 ? u.S * u.S * u.S : u.S * u.S;
    const int64_t tot = (int64_t)u.n * per;
    if (tot <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_user_contrib, dim3((unsigned)((tot + BLOCK - 1) / BLOCK)), dim3(BLOCK), 0, s, u, keys, vals,
                       contrib);
    return hipGetLastError();
}
// one thread per run of equal keys (a grid point): q += c_1, += c_2, ... in list order
__global__ __launch_bounds__(BLOCK) void k_user_segsum(UserDesc u, const unsigned* skeys, const int* svals,
                                                       const double* contrib, int nc) {
    const int e = blockIdx.x * BLOCK + threadIdx.x;
    if (e >= nc || skeys[e] == 0xffffffffu || (e > 0 && skeys[e - 1] == skeys[e])) return;
    double* q = u.cd.u + skeys[e];
    double v = *q;
    for (int j = e; j < nc && skeys[j] == skeys[e]; ++j) v = v + contrib[svals[j]];
    *q = v;
}
hipError_t launch_user_segsum(const UserDesc& u, const unsigned* skeys, const int* svals, const double* contrib,
                              int nc, hipStream_t s) {
    if (nc <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_user_segsum, dim3((nc + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, s, u, skeys, svals, contrib, nc);
    return hipGetLastError();
}

}  // namespace ibtk_le
