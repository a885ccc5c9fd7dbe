// le_sweep.hip -- the 3-D hot path on CDNA4 (gfx950): column binning, and
// interpolation / spreading as z-sweeps over (x,y) columns.  Replaces the
// l-loops of ibtk/src/lagrangian/fortran/lagrangian_interaction3d.f.m4 for every
// kernel function (IB_4 :1258-1522, IB_6 :1851-2255, IB_4_W8 :1532-1850, the
// piecewise kernels :49-971).
//
// Decomposition:
//  * bin: key = (anchor plane z, column, reach band) with columns of COLX x COLY
//    key cells; stable device radix sort; a gather pass writes the sorted
//    marker index and the sorted shifted position X(s)+Xshift(l), fused with
//    the bucket starts.  The sorted list is z-major: one global order.
//  * a sweep work item is (column, z-segment, component).  Everything it reads
//    in its z loop is register-staged one anchor plane ahead with plain loads
//    and put into an LDS ring at the top of the next step.
//  * interp: IWAVES waves per item share the ring of the column's staged region
//    (column + stencil halo) and take alternate anchor planes.  One lane per
//    marker sums its W^3 stencil from the ring in the Fortran loop order (i2,
//    i1, i0), so the value is bitwise the oracle's.
//  * spread: one wave per item owns the column's points in its z-segment, held
//    in an LDS ring of 4 x 4 point tiles.  Planes are loaded (u_old) when the
//    first anchor plane that reaches them comes up and written back when the
//    last one has passed.  The candidates (markers of the 3x3 neighbouring
//    buckets whose stencil reaches the column: 11 contiguous ranges of the
//    sorted list, by band) stream through full 64-lane chunks across anchor
//    planes; each lane computes its candidate's 1-D weights in registers and
//    issues its W^3 adds as LDS f64 atomics (ds_add_f64) in a lane-rotated
//    order that keeps every instruction free of bank conflicts.  Every grid
//    point receives its contributions in a fixed order (staging order, step
//    order, lane order within an instruction): bit-stable from run to run,
//    within rounding of the oracle's sequential l-loop.
#include <hip/hip_runtime.h>

#include <climits>
#include <type_traits>
#include <cstdio>
#include <cstdlib>

#include "le_internal.h"
#include "le_stencil.h"

namespace ibtk_le {

constexpr int SW = 64;  // one wavefront per work item
#ifndef IBTK_LE_DIAG_SPREAD
#define IBTK_LE_DIAG_SPREAD 0  // diagnostic builds only (tools/diag_variants.sh): 1 no adds, 2 trivial weights,
                               // 4 no candidate work, 8 no candidate loads
#endif

// LDS read of one double that the compiler may not merge with its neighbour into a
// ds_read2_b64 (half the rate of two ds_read_b64 on gfx950: interp sweep 10.7 ->
// 9.9 ms on cfg4, round 3)
__device__ __forceinline__ double lds_ld(const double* q) {
    return *(const volatile __attribute__((address_space(3))) double*)q;
}

__device__ __forceinline__ int lane_id() { return __lane_id(); }

// three consecutive doubles (a position record) as one 24-byte load (dwordx4 + dwordx2)
struct D3 {
    double v[3];
};
__device__ __forceinline__ D3 ld3(const double* q) { return *reinterpret_cast<const D3*>(q); }
// Global-memory pointers.  A pointer read from memory (the sorted positions' current
// buffer, Params::sorted_X_ref) is generic to the compiler: its loads become flat_load,
// which may return out of order, so every wait on them is vmcnt(0) lgkmcnt(0) -- it
// waits for every other load and store of the wave as well.  Through an
// address_space(1) pointer they are global_load, and the waits count.
using gdouble = __attribute__((address_space(1))) const double;
__device__ __forceinline__ gdouble* as_global(const double* q) { return (gdouble*)q; }
__device__ __forceinline__ D3 ld3(gdouble* q) {
    D3 r;
#pragma unroll
    for (int d = 0; d < 3; ++d) r.v[d] = q[d];
    return r;
}

// One plane of an Eulerian array as a raw buffer resource (base in SGPRs, a
// 32-bit byte offset per lane): the sweeps' plane loads and stores take one
// VGPR offset and no 64-bit address arithmetic.  Accesses at offsets >= `bytes`
// are dropped by the hardware's range check (loads return 0): the interp stages
// the points outside the array as 0 that way, the spread drops its stores of
// points it does not own.  `base` must be wave-uniform.
constexpr unsigned OFF_NONE = 0x80000000u;  // an offset past every plane (bytes < 2^31)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t plane_rsrc(const void* base, unsigned bytes) {
    const unsigned long long b = reinterpret_cast<unsigned long long>(base);
    const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)b);
    const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(b >> 32));
    void* bp = reinterpret_cast<void*>(((unsigned long long)hi << 32) | lo);
    // dword 3 of a gfx9 buffer resource: 32-bit data format, no swizzle
    return __builtin_amdgcn_make_buffer_rsrc(bp, (short)0, (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}
__device__ __forceinline__ double buf_ld(__amdgpu_buffer_rsrc_t r, unsigned off) {
    return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, (int)off, 0, 0));
}
__device__ __forceinline__ void buf_st(__amdgpu_buffer_rsrc_t r, unsigned off, double v) {
    using V2 = decltype(__builtin_amdgcn_raw_buffer_load_b64(r, 0, 0, 0));
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(V2, v), r, (int)off, 0, 0);
}

// ---------------------------------------------------------------------------
// binning
// ---------------------------------------------------------------------------
// Key cell of a marker relative to the column grid (cell-frame anchor, the same
// rule the stencils use); false if it lies outside the grid (no stencil point
// of it can reach any array).
template <int K>
__device__ __forceinline__ bool col_key_cell(const double* xlo, const double* dx, const int* ilower, const ColGeom& cg,
                                             const double* Xs, int* ka) {
    bool in = true;
#pragma unroll
    for (int d = 0; d < 3; ++d) {
        const double xo = (Xs[d] - xlo[d]) / dx[d];
        if (!(fabs(xo) < 1.0e9)) {  // also catches NaN
            in = false;
            ka[d] = 0;
            continue;
        }
        ka[d] = key_anchor<K>(xo) + ilower[d] - cg.org[d];
        if (ka[d] < 0 || ka[d] >= cg.ext[d]) in = false;
    }
    return in;
}

// The patch of list entry l of a level (binary search of the entry offsets).  A
// wave's entries are mostly of one patch (the sorted order is patch-major): the
// search runs once on the first lane's entry, with scalar loads, and a lane outside
// that patch searches on its own.
__device__ __forceinline__ int entry_patch(const Params& p, int l) {
    auto search = [&](int v) {
        int lo = 0, hi = p.npatch - 1;
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (p.entry_off[mid] <= v) lo = mid;
            else hi = mid - 1;
        }
        return lo;
    };
    const int q = search(__builtin_amdgcn_readfirstlane(l));
    return (p.entry_off[q] <= l && l < p.entry_off[q + 1]) ? q : search(l);
}

// band of a key cell in its column: xb = 0 if its stencil reaches the x-1
// column, 2 if it reaches x+1, else 1; yb likewise; band = 3*xb + yb
template <int K> __device__ __forceinline__ int key_band(int kx, int ky) {
    constexpr int LO = KT<K>::LO, HI = KT<K>::HI;
    static_assert(-1 - LO < COLY - HI, "a stencil must not reach both neighbouring columns");
    const int xl = kx & (COLX - 1), yl = ky % COLY;  // kx, ky >= 0
    const int xb = xl <= -1 - LO ? 0 : (xl >= COLX - HI ? 2 : 1);
    const int yb = yl <= -1 - LO ? 0 : (yl >= COLY - HI ? 2 : 1);
    return 3 * xb + yb;
}

// Bucket key of list entry i at shifted position Xs: (anchor plane, column, band)
// in its patch's bucket range, or nbuckets_total (outside).
template <int K>
// (*zpar, when given: the parity of the entry's z anchor in the frame shifted by -dz/2,
// computed as k_cand_write computes that anchor -- for a stayer, which of the two shifted
// anchors of its key plane it takes)
__device__ __forceinline__ unsigned entry_key(const Params& p, int i, const double* Xs, int* zpar = nullptr) {
    if (p.n_dev && i >= *p.n_dev) return (unsigned)p.nbuckets_total;  // a fixed-capacity list's unused rows
    int ka[3];
    unsigned key = (unsigned)p.nbuckets_total;  // outside
    double zxlo = p.bg.xlo[2];
    if (p.pd) {  // a level: the entry's patch, its frame and its range of buckets
        const PatchDesc& P = p.pd[entry_patch(p, i)];
        zxlo = P.xlo[2];
        if (col_key_cell<K>(P.xlo, p.bg.dx, P.ilower, P.cg, Xs, ka)) {
            const int col = (ka[1] / COLY) * P.cg.ncx + ka[0] / COLX;
            key = (unsigned)(P.bucket_base + (ka[2] * P.cg.ncol + col) * NBAND + key_band<K>(ka[0], ka[1]));
        }
    } else if (col_key_cell<K>(p.bg.xlo, p.bg.dx, p.bg.ilower, p.cg, Xs, ka)) {
        const int col = (ka[1] / COLY) * p.cg.ncx + ka[0] / COLX;
        key = (unsigned)((ka[2] * p.cg.ncol + col) * NBAND + key_band<K>(ka[0], ka[1]));
    }
    if (zpar) {
        const double xo = (Xs[2] - (zxlo - 0.5 * p.bg.dx[2])) * (1.0 / p.bg.dx[2]);
        *zpar = (K == K_IB_4 ? (int)__builtin_rint(xo) : d_nint(xo)) & 1;
    }
    return key;
}

template <int K>
__global__ __launch_bounds__(BLOCK) void k_bin_col(Params p, int n, unsigned* keys, int* vals) {
    const int i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n) return;
    double Xs[3] = {0.0, 0.0, 0.0};
    if (!(p.n_dev && i >= *p.n_dev)) {
        const int s = p.indices ? p.indices[i] : i;
#pragma unroll
        for (int d = 0; d < 3; ++d) Xs[d] = p.Xshift ? p.X[(int64_t)3 * s + d] + p.Xshift[(int64_t)3 * i + d] : p.X[(int64_t)3 * s + d];
    }
    keys[i] = entry_key<K>(p, i, Xs);
    vals[i] = i;
}

// ---------------------------------------------------------------------------
// incremental re-binning (ibtk_le_markers_rebin)
// ---------------------------------------------------------------------------
// The list was binned before: sorted_l / sorted_key hold the order by (key, l)
// of the old positions.  New keys are computed in that order; entries whose key
// did not change ("stayers") keep their relative order, so the new order by
// (key, l) is the stayers' with the changed entries ("movers") inserted.  Per
// bucket b: new count = old + movers in - movers out; a stayer's new position is
// the bucket's new start + the stayers before it in its old bucket + the movers
// into b with a smaller l; a mover's is the new start + the stayers of b with a
// smaller l (a binary search in b's old segment, which is sorted by l) + the
// movers into b with a smaller l.  The movers of a bucket are listed sorted by l.
// Exact: the same order, bucket starts and sorted positions as a fresh binning.
// Nothing is read back to the host; with no movers only k_rekey does work.
//
// The sorted positions live in one of two buffers, xa and xb; *xcur names the
// current one (the sweeps read it through Params::sorted_X_ref).  R1 writes the
// new positions, in the old order, into the other buffer: with nothing moved that
// order is the new one and the commit makes it current; else the scatter reads it
// there (coalesced) and writes the new order into the current buffer.
__device__ __forceinline__ double* rebin_other(double* const* xcur, double* xa, double* xb) {
    return *xcur == xa ? xb : xa;
}
// R1: new keys in the old order; the shifted positions stored at the old sorted
// positions in the other buffer; per-bucket mover counts in/out; the mover flags
// as a bit per entry with per-word counts.
// zbits (closed-form kernels, nullable): the shifted-z anchor parity per sorted position,
// 32 per word (entry_key), compared with the last re-binning's when zst[0] says those are in
// this order (it moved nothing) -- a difference, or none to compare with, sets zst[1] to this
// re-binning's epoch: a split candidate stream (k_cand_write SHZ) must then be rebuilt even
// if nothing moved.  Block 0 also clears the words past the last (mbits / wcnt[nw]) and the
// long-list queue (nbig) the later kernels count on.
template <int K>
__global__ __launch_bounds__(BLOCK) void k_rekey(Params p, int n, const unsigned* kold, const int* sl,
                                                 double* const* xcur, double* xa, double* xb, unsigned* mbits,
                                                 int* wcnt, int* cin, int* cout, unsigned* zbits, int* zst, int epoch,
                                                 int nw, int* nbig) {
    __shared__ double sx[3 * BLOCK];
    const int e0 = blockIdx.x * BLOCK;
    const int e = e0 + threadIdx.x;
    if (blockIdx.x == 0 && threadIdx.x == 0) {  // (a wave ending at word nw writes it 0 as well)
        mbits[nw] = 0u;
        wcnt[nw] = 0;
        *nbig = 0;
    }
    bool mv = false;
    int zp = 0;
    // the last parities of the wave's two words and their state, loaded ahead of the
    // gather (their latency hidden behind it, not added before the block's barrier)
    unsigned zo0 = 0, zo1 = 0;
    int zv = 0;
    if (zbits && (threadIdx.x & 63) == 0 && e < n) {
        zo0 = zbits[e >> 5];
        zo1 = zbits[(e >> 5) + 1];
        zv = zst[0];
    }
    if (e < n) {
        const int l = sl[e];
        const int s = p.indices ? p.indices[l] : l;
        const D3 x = ld3(p.X + (int64_t)3 * s);  // as k_gather_col (a fixed-capacity list's rows all exist)
        double Xs[3];
#pragma unroll
        for (int d = 0; d < 3; ++d) Xs[d] = p.Xshift ? x.v[d] + p.Xshift[(int64_t)3 * l + d] : x.v[d];  // (no + 0.0: X bit for bit)
        const unsigned k = entry_key<K>(p, l, Xs, zbits ? &zp : nullptr);
        const unsigned ko = kold[e];
        mv = k != ko;
        if (mv) {
            atomicAdd(cin + k, 1);
            atomicAdd(cout + ko, 1);
        }
#pragma unroll
        for (int d = 0; d < 3; ++d) sx[3 * threadIdx.x + d] = Xs[d];
    }
    const unsigned long long bal = __ballot(mv);
    if ((threadIdx.x & 63) == 0 && e < n) {  // words e/32, e/32 + 1 (the second may be the zero sentinel)
        const int w = e >> 5;
        mbits[w] = (unsigned)bal;
        mbits[w + 1] = (unsigned)(bal >> 32);
        wcnt[w] = __popc((unsigned)bal);
        wcnt[w + 1] = __popc((unsigned)(bal >> 32));
    }
    if (zbits) {
        const unsigned long long zb = __ballot(zp != 0);
        if ((threadIdx.x & 63) == 0 && e < n) {
            const int w = e >> 5;
            const bool same = zv != 0 && zo0 == (unsigned)zb && zo1 == (unsigned)(zb >> 32);
            zbits[w] = (unsigned)zb;
            zbits[w + 1] = (unsigned)(zb >> 32);
            if (!same) zst[1] = epoch;
        }
    }
    __syncthreads();
    const int cnt = 3 * min(BLOCK, n - e0);
    double* out = rebin_other(xcur, xa, xb) + (int64_t)3 * e0;
    for (int i = threadIdx.x; 2 * i < cnt; i += BLOCK) {
        if (2 * i + 1 < cnt) {
            double2 v;
            v.x = sx[2 * i];
            v.y = sx[2 * i + 1];
            *reinterpret_cast<double2*>(out + 2 * i) = v;
        } else {
            out[2 * i] = sx[2 * i];
        }
    }
}

// R1b (something moved): copies of the old l and the new keys for the scatter,
// which overwrites the sorted arrays (a stayer's new key is its old one; a mover's
// is computed again from its new position, which R1 left in the other buffer)
constexpr int RB_GRID = 4096;  // grid-stride kernels of the re-binning's tail
template <int K>
__global__ __launch_bounds__(BLOCK) void k_rebin_copy(Params p, int n, const int* T, const unsigned* mbits,
                                                      const unsigned* kold, const int* sl, double* const* xcur,
                                                      double* xa, double* xb, unsigned* knew, int* lold, int* zst) {
    // the parities k_rekey wrote are in the new order iff nothing moved
    if (zst && blockIdx.x == 0 && threadIdx.x == 0) zst[0] = *T == 0 ? 1 : 0;
    if (*T == 0) return;
    const double* xo = rebin_other(xcur, xa, xb);
    for (int e = blockIdx.x * BLOCK + threadIdx.x; e < n; e += gridDim.x * BLOCK) {
        const int l = sl[e];
        lold[e] = l;
        unsigned k = kold[e];
        if ((mbits[e >> 5] >> (e & 31)) & 1u) {
            double Xs[3];
#pragma unroll
            for (int d = 0; d < 3; ++d) Xs[d] = xo[(int64_t)3 * e + d];
            k = entry_key<K>(p, l, Xs);
        }
        knew[e] = k;
    }
}

// movers before entry x (0 <= x <= n): word prefix + the word's lower bits
__device__ __forceinline__ int movers_before(const unsigned* mbits, const int* wpre, int x) {
    const int w = x >> 5, b = x & 31;
    return wpre[w] + __popc(mbits[w] & ((1u << b) - 1u));
}
// first position in [lo, hi) of the l-sorted v whose value is >= l
__device__ __forceinline__ int lower_bound_l(const int* v, int lo, int hi, int l) {
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (v[mid] < l) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// Every kernel after k_rekey returns at once when nothing moved (the mover count,
// wpre[nw], is read on the device): a stationary list costs k_rekey and a scan of
// the per-word counts.
//
// R2: per bucket b (0 .. nb + 1; cin / cout[nb + 1] stay 0), the exclusive prefixes of
// d = cin - cout (the shift of b's start) and of cin (b's offset in the movers' list),
// in three phases over blocks of RB_BLK buckets: block sums, a scan of the block sums
// by one workgroup, the blocks' own scans.  ns[b] = os[b] + prefix(d)[b].
constexpr int RB_IPT = 8, RB_BLK = BLOCK * RB_IPT;
// v[i] = a[b0 + i] for b0 + i <= last, else 0 (b0 a multiple of 8: two 16-byte loads)
__device__ __forceinline__ void rb_load8(const int* a, long b0, long last, int* v) {
    if (b0 + 7 <= last) {
        const int4 x = *reinterpret_cast<const int4*>(a + b0), y = *reinterpret_cast<const int4*>(a + b0 + 4);
        v[0] = x.x, v[1] = x.y, v[2] = x.z, v[3] = x.w, v[4] = y.x, v[5] = y.y, v[6] = y.z, v[7] = y.w;
    } else {
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = b0 + i <= last ? a[b0 + i] : 0;
    }
}
// a[b0 + i] = v[i] for b0 + i <= last
__device__ __forceinline__ void rb_store8(int* a, long b0, long last, const int* v) {
    if (b0 + 7 <= last) {
        *reinterpret_cast<int4*>(a + b0) = make_int4(v[0], v[1], v[2], v[3]);
        *reinterpret_cast<int4*>(a + b0 + 4) = make_int4(v[4], v[5], v[6], v[7]);
    } else {
#pragma unroll
        for (int i = 0; i < 8; ++i)
            if (b0 + i <= last) a[b0 + i] = v[i];
    }
}
static_assert(RB_IPT == 8, "rb_load8 / rb_store8");
__global__ __launch_bounds__(BLOCK) void k_rebin_bsum(int nb, const int* cin, const int* cout, const int* T,
                                                      int2* bsum) {
    if (*T == 0) return;
    __shared__ int sd[BLOCK], sc[BLOCK];
    const long b0 = (long)blockIdx.x * RB_BLK + (long)threadIdx.x * RB_IPT;
    int vi[RB_IPT], vo[RB_IPT];
    rb_load8(cin, b0, nb + 1, vi);
    rb_load8(cout, b0, nb + 1, vo);
    int d = 0, c = 0;
#pragma unroll
    for (int i = 0; i < RB_IPT; ++i) {
        d += vi[i] - vo[i];
        c += vi[i];
    }
    sd[threadIdx.x] = d;
    sc[threadIdx.x] = c;
    __syncthreads();
    for (int w = BLOCK / 2; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) {
            sd[threadIdx.x] += sd[threadIdx.x + w];
            sc[threadIdx.x] += sc[threadIdx.x + w];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) bsum[blockIdx.x] = make_int2(sd[0], sc[0]);
}
// one workgroup: bsum[i] := exclusive prefix over the blocks
__global__ __launch_bounds__(BLOCK) void k_rebin_btop(int nblk, const int* T, int2* bsum) {
    if (*T == 0) return;
    __shared__ int sd[BLOCK], sc[BLOCK];
    const int per = (nblk + BLOCK - 1) / BLOCK, i0 = (int)threadIdx.x * per;
    int d = 0, c = 0;
    for (int i = i0; i < min(i0 + per, nblk); ++i) {
        d += bsum[i].x;
        c += bsum[i].y;
    }
    sd[threadIdx.x] = d;
    sc[threadIdx.x] = c;
    __syncthreads();
    if (threadIdx.x == 0) {  // exclusive prefix of the BLOCK thread sums
        int ad = 0, ac = 0;
        for (int t = 0; t < BLOCK; ++t) {
            const int vd = sd[t], vc = sc[t];
            sd[t] = ad;
            sc[t] = ac;
            ad += vd;
            ac += vc;
        }
    }
    __syncthreads();
    d = sd[threadIdx.x];
    c = sc[threadIdx.x];
    for (int i = i0; i < min(i0 + per, nblk); ++i) {
        const int2 v = bsum[i];
        bsum[i] = make_int2(d, c);
        d += v.x;
        c += v.y;
    }
}
__global__ __launch_bounds__(BLOCK) void k_rebin_bapply(int nb, const int* cin, const int* cout, const int* os,
                                                        const int* T, const int2* bsum, int* ns, int* mstart) {
    if (*T == 0) return;
    __shared__ int sd[BLOCK], sc[BLOCK];
    const long b0 = (long)blockIdx.x * RB_BLK + (long)threadIdx.x * RB_IPT;
    int vd[RB_IPT], vc[RB_IPT], vo[RB_IPT], d = 0, c = 0;
    rb_load8(cin, b0, nb + 1, vc);
    rb_load8(cout, b0, nb + 1, vo);
#pragma unroll
    for (int i = 0; i < RB_IPT; ++i) {
        vd[i] = vc[i] - vo[i];
        d += vd[i];
        c += vc[i];
    }
    sd[threadIdx.x] = d;
    sc[threadIdx.x] = c;
    __syncthreads();
    for (int w = 1; w < BLOCK; w <<= 1) {  // inclusive scan of the thread sums
        const int ad = (int)threadIdx.x >= w ? sd[threadIdx.x - w] : 0;
        const int ac = (int)threadIdx.x >= w ? sc[threadIdx.x - w] : 0;
        __syncthreads();
        sd[threadIdx.x] += ad;
        sc[threadIdx.x] += ac;
        __syncthreads();
    }
    d = bsum[blockIdx.x].x + sd[threadIdx.x] - d;  // exclusive: the block's and this thread's offsets
    c = bsum[blockIdx.x].y + sc[threadIdx.x] - c;
    int vs[RB_IPT], vn[RB_IPT], vm[RB_IPT];
    rb_load8(os, b0, nb, vs);
#pragma unroll
    for (int i = 0; i < RB_IPT; ++i) {
        vn[i] = vs[i] + d;
        vm[i] = c;
        d += vd[i];
        c += vc[i];
    }
    rb_store8(ns, b0, nb, vn);
    rb_store8(mstart, b0, nb + 1, vm);
}

// R3: every mover appends its l to its new bucket's list (mstart: exclusive prefix
// of the in-counts); the counts are consumed (cin back to 0, cout reset), so the
// next re-binning starts from zeros without a memset.  One thread per word of flags.
__global__ __launch_bounds__(BLOCK) void k_rebin_append(int n, int nw, const unsigned* mbits, const unsigned* knew,
                                                        const unsigned* kold, const int* lold, const int* mstart,
                                                        int* cin, int* cout, int* mlist) {
    const int w = blockIdx.x * BLOCK + threadIdx.x;
    if (w >= nw) return;
    unsigned bits = mbits[w];
    while (bits) {
        const int e = 32 * w + __ffs(bits) - 1;
        bits &= bits - 1;
        const unsigned b = knew[e];
        const int j = atomicSub(cin + b, 1) - 1;
        mlist[mstart[b] + j] = lold[e];
        cout[kold[e]] = 0;
    }
}
// Each bucket's mover list sorted by l: lists of up to 32 by one thread (insertion
// sort); longer ones are queued for k_rebin_sort_big
constexpr int REBIN_SMALL = 32;
__global__ __launch_bounds__(BLOCK) void k_rebin_sort_small(int nb, const int* T, const int* mstart, int* mlist,
                                                            int* nbig, int* big) {
    if (*T == 0) return;
    for (int b = blockIdx.x * BLOCK + threadIdx.x; b <= nb; b += gridDim.x * BLOCK) {
        const int lo = mstart[b], k = mstart[b + 1] - lo;
        if (k < 2) continue;
        if (k > REBIN_SMALL) {
            big[atomicAdd(nbig, 1)] = b;
            continue;
        }
        int* v = mlist + lo;
        for (int i = 1; i < k; ++i) {
            const int x = v[i];
            int j = i - 1;
            while (j >= 0 && v[j] > x) {
                v[j + 1] = v[j];
                --j;
            }
            v[j + 1] = x;
        }
    }
}
// Long lists (clustered markers crossing a plane together): the rank of every
// entry is the count of smaller l in its list (l are distinct), counted through
// LDS by a workgroup per list; the sorted list goes to scratch, copied back by
// k_rebin_copy_big.
__global__ __launch_bounds__(BLOCK) void k_rebin_sort_big(const int* nbig, const int* big, const int* mstart,
                                                          const int* mlist, int* scratch) {
    __shared__ int sh[BLOCK];
    const int nb_ = *nbig;
    for (int i = blockIdx.x; i < nb_; i += gridDim.x) {
        const int b = big[i];
        const int base = mstart[b], k = mstart[b + 1] - base;
        for (int t = 0; t < k; t += BLOCK) {
            const bool own = t + (int)threadIdx.x < k;
            const int x = own ? mlist[base + t + threadIdx.x] : INT_MAX;
            int rank = 0;
            for (int c = 0; c < k; c += BLOCK) {
                __syncthreads();
                sh[threadIdx.x] = c + (int)threadIdx.x < k ? mlist[base + c + threadIdx.x] : INT_MAX;
                __syncthreads();
                const int m = min(BLOCK, k - c);
                for (int j = 0; j < m; ++j) rank += sh[j] < x;
            }
            if (own) scratch[base + rank] = x;
        }
    }
}
__global__ __launch_bounds__(BLOCK) void k_rebin_copy_big(const int* nbig, const int* big, const int* mstart,
                                                          const int* scratch, int* mlist) {
    const int nb_ = *nbig;
    for (int i = blockIdx.x; i < nb_; i += gridDim.x) {
        const int b = big[i];
        const int base = mstart[b], k = mstart[b + 1] - base;
        for (int t = threadIdx.x; t < k; t += BLOCK) mlist[base + t] = scratch[base + t];
    }
}

// old entry e's new sorted position, returned; l, key and marker index written
// there, its shifted position (R1's, in the other buffer xo) into x
__device__ __forceinline__ int rebin_place(const Params& p, int e, int n, int nb, const unsigned* mbits,
                                           const int* wpre, const unsigned* knew, const int* lold, const int* os,
                                           const int* ns, const int* mstart, const int* mlist, const double* xo,
                                           int* sorted_l, unsigned* sorted_key, int* sorted_s, double* x) {
    const int l = lold[e];
    const int b = (int)knew[e];
    const int ob = os[b], oe = b < nb ? os[b + 1] : n;
    const int mb0 = movers_before(mbits, wpre, ob);
    int pos;
    if ((mbits[e >> 5] >> (e & 31)) & 1u) {
        const int lb = lower_bound_l(lold, ob, oe, l);  // old entries of b with a smaller l
        pos = ns[b] + (lb - ob) - (movers_before(mbits, wpre, lb) - mb0);
    } else {
        pos = ns[b] + (e - ob) - (movers_before(mbits, wpre, e) - mb0);
    }
    pos += lower_bound_l(mlist, mstart[b], mstart[b + 1], l) - mstart[b];
    sorted_l[pos] = l;
    sorted_key[pos] = (unsigned)b;
    sorted_s[pos] = p.indices ? p.indices[l] : l;
#pragma unroll
    for (int d = 0; d < 3; ++d) x[d] = xo[(int64_t)3 * e + d];
    return pos;
}
// R4 (only when something moved: wpre[nw] is the mover count): every entry to its
// new sorted position; the sorted arrays rewritten there, the positions read from
// the other buffer in the old order and written into the current one.  The
// positions leave through LDS: a block's records go
// out as consecutive doubles of consecutive records (a stayer run's new positions
// are consecutive), not as a wave's 8-byte stores at a 24-byte stride, which write
// every 64-byte piece three times.
constexpr int RB_U = 1;
__global__ __launch_bounds__(BLOCK) void k_rebin_scatter(Params p, int n, int nb, const unsigned* __restrict__ mbits,
                                                         const int* __restrict__ wpre, int nw,
                                                         const unsigned* __restrict__ knew,
                                                         const int* __restrict__ lold, const int* __restrict__ os,
                                                         const int* __restrict__ ns, const int* __restrict__ mstart,
                                                         const int* __restrict__ mlist, int* __restrict__ sorted_l,
                                                         unsigned* __restrict__ sorted_key, int* __restrict__ sorted_s,
                                                         double* const* xcur, double* xa, double* xb) {
    if (wpre[nw] == 0) return;
    double* const sorted_X = *xcur;
    const double* const xo = rebin_other(xcur, xa, xb);
    __shared__ double sx[3 * RB_U * BLOCK];
    __shared__ int sp[RB_U * BLOCK];
    for (int e0 = blockIdx.x * RB_U * BLOCK; e0 < n; e0 += gridDim.x * RB_U * BLOCK) {
#pragma unroll
        for (int u = 0; u < RB_U; ++u) {
            const int i = u * BLOCK + threadIdx.x, e = e0 + i;
            if (e < n) {
                double x[3];
                sp[i] = rebin_place(p, e, n, nb, mbits, wpre, knew, lold, os, ns, mstart, mlist, xo, sorted_l,
                                    sorted_key, sorted_s, x);
#pragma unroll
                for (int d = 0; d < 3; ++d) sx[3 * i + d] = x[d];
            }
        }
        __syncthreads();
        const int cnt = 3 * min(RB_U * BLOCK, n - e0);
        for (int i = threadIdx.x; i < cnt; i += BLOCK) {
            const int r = i / 3;
            sorted_X[(int64_t)3 * sp[r] + (i - 3 * r)] = sx[i];
        }
        __syncthreads();
    }
}
// the new bucket starts in place when something moved; else the other buffer,
// which holds the new positions in the unchanged order, becomes current
__global__ __launch_bounds__(BLOCK) void k_rebin_commit(int nb, const int* T, const int* ns, int* plane_start,
                                                        double** xcur, double* xa, double* xb, int* order_gen) {
    if (*T == 0) {
        if (blockIdx.x == 0 && threadIdx.x == 0) *xcur = rebin_other(xcur, xa, xb);
        return;
    }
    if (order_gen && blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(order_gen, 1);  // a new order
    for (int b = blockIdx.x * BLOCK + threadIdx.x; b <= nb; b += gridDim.x * BLOCK) plane_start[b] = ns[b];
}
// *xcur := x (a fresh binning gathered the positions into x)
__global__ void k_set_xcur(double** xcur, double* x) { *xcur = x; }
hipError_t launch_set_xcur(double** xcur, double* x, hipStream_t s) {
    hipLaunchKernelGGL(k_set_xcur, dim3(1), dim3(1), 0, s, xcur, x);
    return hipGetLastError();
}

// Per sorted entry e: the marker index and the shifted position (coalesced for
// the sweeps), fused with the bucket starts: the first entry of every non-empty
// bucket writes its index into first[] (keys >= nbuckets: binned outside, bucket
// nbuckets), which k_bucket_init set to n; a suffix-min scan over first[] then
// gives every bucket's start (launch_suffix_min).  n > 0.
// The block's 3 BLOCK positions leave through LDS as 16-byte stores (a wave's
// 8-byte stores at a 24-byte stride would write each cache line in thirds).
template <int K>
__global__ __launch_bounds__(BLOCK) void k_gather_col(Params p, int n, int* sorted_s, double* sorted_X,
                                                      const unsigned* skeys, int nbuckets, int* first) {
    __shared__ double sx[3 * BLOCK];
    const int e0 = blockIdx.x * BLOCK;
    const int e = e0 + threadIdx.x;
    if (e < n) {
        const int bi = (int)min(skeys[e], (unsigned)nbuckets);
        if (e == 0 || bi != (int)min(skeys[e - 1], (unsigned)nbuckets)) first[bi] = e;
        const int l = p.sorted_l[e];
        const int s = p.indices ? p.indices[l] : l;
        sorted_s[e] = s;
        const D3 x = ld3(p.X + (int64_t)3 * s);  // one 24-byte record per lane
#pragma unroll
        for (int d = 0; d < 3; ++d) sx[3 * threadIdx.x + d] = p.Xshift ? x.v[d] + p.Xshift[(int64_t)3 * l + d] : x.v[d];
    }
    __syncthreads();
    const int cnt = 3 * min(BLOCK, n - e0);  // doubles this block writes
    double* out = sorted_X + (int64_t)3 * e0;  // 16-byte aligned: 3 BLOCK e0 doubles in
    for (int i = threadIdx.x; 2 * i < cnt; i += BLOCK) {
        if (2 * i + 1 < cnt) {
            double2 v;
            v.x = sx[2 * i];
            v.y = sx[2 * i + 1];
            *reinterpret_cast<double2*>(out + 2 * i) = v;
        } else {
            out[2 * i] = sx[2 * i];
        }
    }
}

// the current sorted positions of a 3-D binning (Params::sorted_X_ref: xa or xb of
// the re-binning), read once per kernel
__device__ __forceinline__ gdouble* cur_sorted_X(const Params& p) {
    typedef const double* dptr;
    if (!p.sorted_X_ref) return as_global(p.sorted_X);
    return as_global(*(const __attribute__((address_space(1))) dptr*)p.sorted_X_ref);
}

// ---------------------------------------------------------------------------
// work items
// ---------------------------------------------------------------------------
// Items are (segment, column, component), component fastest.  The heavy items
// (k_item_counts: clustered markers, p.nitems[1] of them) head the table and
// take the first blocks, dealt round-robin over the XCDs, so that they start
// first and the light ones fill in around them.  The light items go to the XCDs
// in blocks of B table entries (block j to XCD j mod 8), so the three
// components of a column and its x-neighbours run on one XCD at about the same
// time and share marker data and halo planes through its L2.  The item count
// is read on the device (the grid is an upper bound of it).
constexpr int XCD_BLOCK = 8;  // table entries per block of items dealt to one XCD
__device__ __forceinline__ int sweep_item(const Params& p, int per_entry) {
    const int nt = p.nitems[0] * per_entry, nh = p.nitems[1] * per_entry;
    const int b = blockIdx.x;
    const int h8 = (nh + 7) & ~7;
    if (b < h8) return b < nh ? b : -1;
    const int bl = b - h8, nl = nt - nh;
    // ctx_tune xcd_block: 1 = round-robin, -1 = one contiguous range per XCD (the
    // round-1 order).  Contiguous ranges give one XCD a whole z-layer of a
    // level's patches -- a sheet of markers: blocks take cfg5 from 1.74e9 to
    // 1.96e9 marker-ops/s (spread sweep 4.32 -> 3.41 ms); on cfg4 blocks of 8
    // keep the x-neighbour columns' shared halo lines in one L2 (profiles/r02z).
    const int B = p.tune.xcd_block != 0 ? p.tune.xcd_block : XCD_BLOCK;
    if (B > 0) {
        const int Bi = B * per_entry;  // items per block
        const int k = bl >> 3, x = bl & 7;
        const int it = ((k / Bi) * 8 + x) * Bi + (k % Bi);
        return it < nl ? nh + it : -1;
    }
    const int per = (nl + 7) >> 3;
    if ((bl >> 3) >= per) return -1;
    const int it = (bl & 7) * per + (bl >> 3);
    return it < nl ? nh + it : -1;
}

// Work item -> (component c, table entry t): component fastest, so the three
// components of a column run on one XCD at about the same time (their Q
// stores fill the same AoS lines).  The table (k_item_write) lists the
// (column, owned planes [p0, p1)) of every item, segment-major.
__device__ __forceinline__ void item_decode(const Params& p, int it, int& c, SweepItem& si) {
    const int t = it / p.ncomp;
    c = it - t * p.ncomp;
    si = p.items[t];
}

// bucket index of (anchor plane a, column col, band) in the patch's table
__device__ __forceinline__ int bucket(const ColGeom& cg, int a, int col, int band) {
    return (a * cg.ncol + col) * NBAND + band;
}

// The item's patch: its column grid, the component's array and its bucket table.
template <bool LVL>
__device__ __forceinline__ void item_patch(const Params& p, const SweepItem& si, int c, ColGeom& cg, CompDesc& cd,
                                           const int*& bs) {
    if constexpr (LVL) {
        const PatchDesc& P = p.pd[si.patch];
        cg = P.cg;
        cd = P.comp[c];
        bs = p.plane_start + P.bucket_base;
    } else {
        cg = p.cg;
        cd = p.comp[c];
        bs = p.plane_start;
    }
}

// ---------------------------------------------------------------------------
// diagnostics
// ---------------------------------------------------------------------------
// Phase clocks (s_memtime per work item, IBTK_LE_STAMPS=1 at run time) exist
// only in builds with -DIBTK_LE_CLOCKS=1: their 64-bit accumulators would
// otherwise hold 14 SGPRs through the sweep loop.
#ifndef IBTK_LE_CLOCKS
#define IBTK_LE_CLOCKS 0
#endif
#if IBTK_LE_CLOCKS
struct Clk {
    unsigned long long t = 0, acc[6] = {0, 0, 0, 0, 0, 0};
    bool on = false;
    __device__ __forceinline__ void start(bool enable) {
        on = enable;
        if (on) t = __builtin_amdgcn_s_memtime();
    }
    __device__ __forceinline__ void lap(int ph) {
        if (on) {
            const unsigned long long u = __builtin_amdgcn_s_memtime();
            acc[ph] += u - t;
            t = u;
        }
    }
    __device__ __forceinline__ void flush(const Params& p, int it) {
        if (on && lane_id() == 0)
            for (int k = 0; k < 6; ++k) p.stamps[(int64_t)it * 8 + k] = acc[k];
    }
};
#else
struct Clk {
    __device__ __forceinline__ void start(bool) {}
    __device__ __forceinline__ void lap(int) {}
    __device__ __forceinline__ void flush(const Params&, int) {}
};
#endif

// ---------------------------------------------------------------------------
// interpolation
// ---------------------------------------------------------------------------
constexpr int IWAVES = 4;  // waves per interp work item (one LDS ring)

template <int K> struct ISh {
    using T = KT<K>;
    static constexpr int W = T::W, LO = T::LO, HI = T::HI, FAM = T::FAM;
    static constexpr int RX = COLX + HI - LO, RY = COLY + HI - LO;  // staged plane: column + stencil halo
    static constexpr int NS = HI - LO + 1;                          // planes an anchor plane reads (a+LO .. a+HI)
    static constexpr int NSL = NS + IWAVES - 1;                     // ring slots: the planes IWAVES anchors read
    static constexpr int PV = RX * RY;
    static constexpr int NPT = (PV + SW - 1) / SW;                  // staged points per lane and plane
    // ring slot stride: a multiple of 32 doubles, so a point's LDS bank class
    // (f64 index mod 32) does not depend on its plane
    static constexpr int PVP = (PV + 31) / 32 * 32;
};

template <int K> __device__ __forceinline__ int islot(int prel) {
    using S = ISh<K>;
    return (int)((unsigned)(prel - S::LO) % (unsigned)S::NSL);  // prel >= LO
}

template <int K>
__device__ __forceinline__ double interp_marker(const Params& p, const CompDesc& cd, const double* ring, int gx0,
                                                int gy0, int zorg, int a, const double* Xs, int s) {
    using S = ISh<K>;
    constexpr int W = S::W, FAM = S::FAM, RX = S::RX, PV = S::PVP;  // PV: ring slot stride
    St<W> st[3];
#pragma unroll
    for (int d = 0; d < 3; ++d) {
        const double Xraw = (FAM == 2) ? p.X[(int64_t)3 * s + d] : Xs[d];
        stencil1d<K>(Xs[d], Xraw, cd.xlo[d], p.bg.dx[d], cd.ilower[d], cd.lo[d], cd.hi[d], d == cd.axis, p.K6, st[d]);
    }
    const int ox = st[0].icl - gx0, oy = st[1].icl - gy0, oz = st[2].icl - zorg;
    // binning invariant: the points read lie in the staged column region and
    // ring (FAM 0 reads all W per dim, clipped ones as staged zeros)
    bool ok;
    if constexpr (FAM == 0) {
        // (a cell-frame dim's last staged index is not loaded: k_interp_sweep's poff)
        ok = ox >= 0 && ox + W <= RX - cd.xcell && oy >= 0 && oy + W <= S::RY - cd.ycell && oz >= a + S::LO &&
             oz + W - 1 <= a + S::HI;
    } else {
        bool empty = false;
#pragma unroll
        for (int d = 0; d < 3; ++d) empty = empty || st[d].ist > st[d].isp;
        if (empty) return 0.0;
        ok = ox + st[0].ist >= 0 && ox + st[0].isp < RX && oy + st[1].ist >= 0 && oy + st[1].isp < S::RY &&
             oz + st[2].ist >= a + S::LO && oz + st[2].isp <= a + S::HI;
    }
    if (!ok) {
        atomicOr(p.err, 1);
        return 0.0;
    }
    double acc = 0.0;
    if constexpr (FAM == 3) {
        acc = ring[islot<K>(oz) * PV + oy * RX + ox];
    } else if constexpr (FAM == 0) {
        // Clipped points (outside the ghost box) are staged as 0: acc + (w*wyz)*0
        // == acc bit for bit (acc is never -0), so the clipped sum of
        // f.m4:1366-1382 needs no per-point branch.  The reads of a block of R
        // stencil rows (R W ~ 16 values) go out back to back before the block is
        // summed, so one LDS latency is exposed per block rather than one per
        // pair of reads (the sum itself stays the Fortran's sequential chain).
        const double* base = ring + oy * RX + ox;
        constexpr int R = W <= 4 ? W : (W <= 6 ? 3 : 2);  // rows per block; divides W
#pragma unroll
        for (int i2 = 0; i2 < W; ++i2) {
            const double* pl = base + islot<K>(oz + i2) * PV;
#pragma unroll
            for (int r0 = 0; r0 < W; r0 += R) {
                double v[R * W];
#pragma unroll
                for (int r = 0; r < R; ++r)
#pragma unroll
                    for (int i0 = 0; i0 < W; ++i0)
                        v[r * W + i0] = lds_ld(&pl[(r0 + r) * RX + i0]);
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const double wyz = st[1].w[r0 + r] * st[2].w[i2];  // f.m4:1349-1353
#pragma unroll
                    for (int i0 = 0; i0 < W; ++i0) {
                        const double wt = st[0].w[i0] * wyz;
                        acc = acc + wt * v[r * W + i0];  // f.m4:1375
                    }
                }
            }
        }

    } else {
        // piecewise kernels: weights outside [ist, isp] are 0 and the index is
        // clamped into the stencil's valid range, acc + 0*u == acc.
        double w[3][W];
        int o[3][W];
#pragma unroll
        for (int d = 0; d < 3; ++d) {
#pragma unroll
            for (int i = 0; i < W; ++i) {
                const bool in = i >= st[d].ist && i <= st[d].isp;
                w[d][i] = in ? st[d].w[i] : 0.0;
                o[d][i] = min(max(i, st[d].ist), st[d].isp);
            }
        }
#pragma unroll
        for (int i2 = 0; i2 < W; ++i2) {
            const double* pl = ring + islot<K>(oz + o[2][i2]) * PV + oy * RX + ox;
#pragma unroll
            for (int i1 = 0; i1 < W; ++i1) {
#pragma unroll
                for (int i0 = 0; i0 < W; ++i0)
                    acc = acc + w[0][i0] * w[1][i1] * w[2][i2] * pl[o[1][i1] * RX + o[0][i0]];  // f.m4:545-548
            }
        }
    }
    return acc;
}

// Interpolation work item = (segment, column, component), one workgroup of
// IWAVES waves sharing one LDS ring (more waves per CU for the same LDS: the
// per-marker sum is a dependent chain in the Fortran order, so the latency
// wants waves).  The waves take the item's anchor planes in groups of IWAVES:
// the ring holds planes a+LO .. a+IWAVES-1+HI.  Per group: barrier (the
// previous group's reads are done), wave w puts one new plane (a+w+HI) into
// the slot a retired plane left, barrier, each wave prefetches its next plane
// and markers into registers (plain loads) and sums its chunks of the group's
// pooled markers.  Points outside the component's array are staged as 0.  One
// lane per marker sums its W^3 stencil from the ring (Fortran loop order,
// bitwise the oracle's).
// ibtk_le_level_fill_interp's record per (component, patch): 27 suppliers {window offset,
// mapped}, then the window base (lo, hi 32 bits) and its length in bytes
constexpr int LVL_REC = 32;
// the plane-independent part of a staged point's offset for class (dx, dy) at plane
// direction dz (k_interp_sweep, LF): the supplier's window offset less its index shift
__device__ __forceinline__ unsigned lvl_class(const int2* tab, int dx, int dy, int dz, int n0, int n1, int n2,
                                              int64_t s1, int64_t s2) {
    const int2 e = tab[dx + 3 * dy + 9 * dz];
    const int64_t shift = e.y ? (int64_t)dx * n0 + (int64_t)dy * n1 * s1 + (int64_t)dz * n2 * s2 : 0;
    return (unsigned)e.x - (unsigned)(8 * shift);
}
// LF: a level with its ghost fill fused in (p.lvl_nbr; a kernel of its own, so that the
// plain level sweep keeps its registers)
template <int K, bool LVL, bool LF = false>
__global__ __launch_bounds__(SW * IWAVES) void k_interp_sweep(Params p) {
    static_assert(LVL || !LF, "the fused fill is a level's");
    using S = ISh<K>;
    constexpr int LO = S::LO, HI = S::HI, RX = S::RX, NPT = S::NPT;
    __shared__ double ring[S::NSL * S::PVP];
    const int it = sweep_item(p, p.ncomp);
    if (it < 0) return;
    int c;
    SweepItem si;
    item_decode(p, it, c, si);
    const int col = si.col;
    const int a0 = si.p0, a1 = si.p1;  // the item's anchor planes
    const int lane = lane_id();
    const int w = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
    ColGeom cg;
    CompDesc cd;
    const int* bs;
    item_patch<LVL>(p, si, c, cg, cd, bs);
    gdouble* const sorted_X = cur_sorted_X(p);
    if (p.zmode) {  // the planes the item reads: a0 + LO .. a1 - 1 + HI
        const bool inner = cg.org[2] + a0 + LO >= p.zlo && cg.org[2] + a1 - 1 + HI <= p.zhi;
        if (inner != (p.zmode == 1)) return;
    }
    {
        bool any = false;  // the same answer in every wave
        for (int a = a0 + lane; a < a1; a += SW) any = any || bs[bucket(cg, a, col, NBAND)] > bs[bucket(cg, a, col, 0)];
        if (!__any(any)) return;
    }
    const int cx = col % cg.ncx, cy = col / cg.ncx;
    const int gx0 = cg.org[0] + cx * COLX + LO, gy0 = cg.org[1] + cy * COLY + LO;
    const int zorg = cg.org[2];
    const int nlast = p.nsorted - 1;
    // the lane's staged points q = lane + 64 k: array offsets (clamped) and
    // in-array bits (x, y)
    // the lane's staged points q = lane + 64 k: byte offsets in a plane through a
    // buffer resource (plane_rsrc); a point outside the array has OFF_NONE, and a
    // plane outside it an empty resource, so their loads return the 0 the
    // clipped stencil points are staged as (no select per point)
    // iper (ibtk_le_fill_interp): a ghost point of the ghost box is read at its periodic
    // image in the periodic dims -- the value the periodic fill would copy there (k_ghost
    // mode 0: every periodic dim wrapped into the patch box); points outside the ghost
    // box stay clipped (staged as 0)
    auto image = [&](int i, int d) {
        if (!p.iper[d] || (i >= cd.ilower[d] && i <= cd.iupper[d])) return i;
        const int n = cd.iupper[d] - cd.ilower[d] + 1;
        int r = (i - cd.ilower[d]) % n;
        return cd.ilower[d] + (r < 0 ? r + n : r);
    };
    // The closed-form kernels (FAM 0) read, in a dim where the component's frame is the keys'
    // (cell) frame, only the staged indices [0, RX - 2] (x) / [0, RY - 2] (y): the stencil of
    // key k spans k + [LO, HI - 1] there (the spread's ZC ring rests on the same fact in z).
    // Such a component's last staged column / row is not loaded (staged as 0, never read).
    const bool xlast = S::FAM == 0 && cd.xcell, ylast = S::FAM == 0 && cd.ycell;
    unsigned poff[NPT];
#pragma unroll
    for (int k = 0; k < NPT; ++k) {
        const int q = min(lane + SW * k, S::PV - 1);
        const int qx = q % RX, qy = q / RX;
        const int gx = gx0 + qx, gy = gy0 + qy;
        const bool in = gx >= cd.lo[0] && gx <= cd.hi[0] && gy >= cd.lo[1] && gy <= cd.hi[1] &&
                        !(xlast && qx == RX - 1) && !(ylast && qy == S::RY - 1);
        poff[k] = in ? 8u * (unsigned)((image(gx, 0) - cd.lo[0]) + (image(gy, 1) - cd.lo[1]) * (int)cd.s1) : OFF_NONE;
    }
    // level fill fused (p.lvl_nbr, LVL only): a staged point outside the patch box is read
    // in the neighbour patch that supplies it.  The staged region crosses at most one face
    // per dim (the host asks for patches at least RX x RY cells), toward (sxd, syd): a
    // point's class is 2 bits (beyond the x face, beyond the y face), and per plane four
    // uniform offsets, one per class, turn its unmapped offset poff[k] into the supplier's
    // (the neighbour's window offset, the -dir n index shift, the plane)
    constexpr bool lfill = LF;
    unsigned lsel = 0;  // bits 2k, 2k+1: the class of point k
    // per plane direction dz and class: the plane-independent part of the class offset
    // (the supplier's window offset, its x/y/z index shift), read once per item
    // (named scalars, not arrays: an array selected by class or plane direction would go to scratch)
    struct Cls {
        unsigned o0, o1, o2, o3;
    };
    Cls ob_m{}, ob_0{}, ob_p{};
    const double* lbase = nullptr;  // the component's level window
    unsigned lspan = 0;
    int sxd = 0, syd = 0;
    if constexpr (LF) {
        {
            sxd = gx0 < cd.ilower[0] ? -1 : (gx0 + RX - 1 >= cd.ilower[0] + p.lvl_n[0] ? 1 : 0);
            syd = gy0 < cd.ilower[1] ? -1 : (gy0 + S::RY - 1 >= cd.ilower[1] + p.lvl_n[1] ? 1 : 0);
            const int2* rec = p.lvl_nbr + ((int64_t)c * p.npatch + si.patch) * LVL_REC;
            const int2* tab = rec + 13;
            const int n0 = p.lvl_n[0], n1 = p.lvl_n[1], n2 = p.lvl_n[2];
            const int64_t s1 = cd.s1, s2 = cd.s2;
            ob_m = Cls{lvl_class(tab, 0, 0, -1, n0, n1, n2, s1, s2), lvl_class(tab, sxd, 0, -1, n0, n1, n2, s1, s2),
                       lvl_class(tab, 0, syd, -1, n0, n1, n2, s1, s2), lvl_class(tab, sxd, syd, -1, n0, n1, n2, s1, s2)};
            ob_0 = Cls{lvl_class(tab, 0, 0, 0, n0, n1, n2, s1, s2), lvl_class(tab, sxd, 0, 0, n0, n1, n2, s1, s2),
                       lvl_class(tab, 0, syd, 0, n0, n1, n2, s1, s2), lvl_class(tab, sxd, syd, 0, n0, n1, n2, s1, s2)};
            ob_p = Cls{lvl_class(tab, 0, 0, 1, n0, n1, n2, s1, s2), lvl_class(tab, sxd, 0, 1, n0, n1, n2, s1, s2),
                       lvl_class(tab, 0, syd, 1, n0, n1, n2, s1, s2), lvl_class(tab, sxd, syd, 1, n0, n1, n2, s1, s2)};
            // the window from the record (an index by component into the kernel arguments would
            // copy them to scratch)
            const int2 wb = rec[27], ws = rec[28];
            lbase = reinterpret_cast<const double*>(((uint64_t)(unsigned)wb.y << 32) | (unsigned)wb.x);
            lspan = (unsigned)ws.x;
#pragma unroll
            for (int k = 0; k < NPT; ++k) {
                const int q = min(lane + SW * k, S::PV - 1);
                const int gx = gx0 + q % RX, gy = gy0 + q / RX;
                const bool bx = gx < cd.ilower[0] || gx >= cd.ilower[0] + p.lvl_n[0];
                const bool by = gy < cd.ilower[1] || gy >= cd.ilower[1] + p.lvl_n[1];
                lsel |= ((bx ? 1u : 0u) | (by ? 2u : 0u)) << (2 * k);
            }
        }
    }
    const int plast = a1 - 1 + HI;  // last plane the item reads
    const unsigned plane_bytes = (unsigned)(8 * cd.s2);
    // relative plane zr -> registers
    auto plane_load = [&](int zr, double* v) __attribute__((always_inline)) {  // (inlined: a call would take p's address)
        const int z0 = zorg + min(zr, plast);
        const bool zin = z0 >= cd.lo[2] && z0 <= cd.hi[2];
        if constexpr (LF) {
            {  // one resource over the component's level window
                const int dz = z0 < cd.ilower[2] ? -1 : (z0 >= cd.ilower[2] + p.lvl_n[2] ? 1 : 0);
                const unsigned zo = (unsigned)(8 * (int64_t)(z0 - cd.lo[2]) * cd.s2);
                // the row of dz by masks (a select chain here becomes a table in scratch)
                const unsigned mm = 0u - (unsigned)(dz < 0), mp = 0u - (unsigned)(dz > 0), m0 = ~(mm | mp);
                const unsigned O0 = ((ob_m.o0 & mm) | (ob_0.o0 & m0) | (ob_p.o0 & mp)) + zo;
                const unsigned O1 = ((ob_m.o1 & mm) | (ob_0.o1 & m0) | (ob_p.o1 & mp)) + zo;
                const unsigned O2 = ((ob_m.o2 & mm) | (ob_0.o2 & m0) | (ob_p.o2 & mp)) + zo;
                const unsigned O3 = ((ob_m.o3 & mm) | (ob_0.o3 & m0) | (ob_p.o3 & mp)) + zo;
                const auto pb = plane_rsrc(lbase, zin ? lspan : 0u);
#pragma unroll
                for (int k = 0; k < NPT; ++k) {
                    const unsigned cl = (lsel >> (2 * k)) & 3u;
                    const unsigned o = (cl & 2u) ? ((cl & 1u) ? O3 : O2) : ((cl & 1u) ? O1 : O0);
                    v[k] = buf_ld(pb, poff[k] == OFF_NONE ? OFF_NONE : poff[k] + o);
                }
                return;
            }
        }
        const int z = zin ? image(z0, 2) : z0;
        const int zc = min(max(z, cd.lo[2]), cd.hi[2]);
        const auto pb = plane_rsrc(cd.u + (int64_t)(zc - cd.lo[2]) * cd.s2, zin ? plane_bytes : 0u);
#pragma unroll
        for (int k = 0; k < NPT; ++k) v[k] = buf_ld(pb, poff[k]);
    };
    auto plane_put = [&](int zr, const double* v) {  // registers -> ring slot
        double* sl = ring + islot<K>(zr) * S::PVP;
#pragma unroll
        for (int k = 0; k < NPT; ++k)
            if (S::PV % SW == 0 || k < NPT - 1 || lane + SW * k < S::PV) sl[lane + SW * k] = v[k];
    };
    struct Mk {
        int s;
        int q;  // the marker whose Q this entry writes (-1: a later duplicate entry does)
        double X[3];
    };
    // LDS barrier of the waves; global loads in flight stay in flight
    auto lds_barrier = [&]() {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
    };

    // The markers of a group's IWAVES anchor planes are pooled and dealt in
    // 64-lane chunks (chunk c to wave c mod IWAVES): the ring holds every plane
    // the group's markers read, so any wave can sum any of them, and about
    // 3.5 chunks per group replace 4 three-quarter-full ones.  Each marker is
    // still summed by one lane in the Fortran order (bitwise unchanged).
    // Group spans: lane k < IWAVES holds the first sorted entry of anchor a+k,
    // lane IWAVES+k its end (loaded a group ahead, read with readlane).
    struct GSpan {
        int beg[IWAVES];
        int pre[IWAVES + 1];
    };
    auto gspan_load = [&](int a) {
        const int k = lane < IWAVES ? lane : min(lane - IWAVES, IWAVES - 1);
        const int ac = min(a + k, cg.nz - 1);
        return bs[bucket(cg, ac, col, lane >= IWAVES && lane < 2 * IWAVES ? NBAND : 0)];
    };
    auto gspan_get = [&](int a, int v, GSpan& gsp) {
        int acc = 0;
#pragma unroll
        for (int k = 0; k < IWAVES; ++k) {
            const int b = __builtin_amdgcn_readlane(v, k);
            const int e = a + k < a1 ? __builtin_amdgcn_readlane(v, IWAVES + k) : b;
            gsp.beg[k] = b;
            gsp.pre[k] = acc;
            acc += e - b;
        }
        gsp.pre[IWAVES] = acc;
    };
    // chunk c of a group: entry 64 c + lane (clamped), with its anchor plane
    auto chunk_load = [&](const GSpan& gsp, int a, int c, Mk& m, int& am) {
        const int tot = gsp.pre[IWAVES];
        const int j = min(SW * c + lane, max(tot - 1, 0));
        int e = gsp.beg[0] + j, k = 0;
#pragma unroll
        for (int q = 1; q < IWAVES; ++q)
            if (j >= gsp.pre[q]) {
                e = gsp.beg[q] + (j - gsp.pre[q]);
                k = q;
            }
        am = a + k;
        e = min(e, nlast);
        m.s = p.sorted_s[e];
        m.q = (p.qdst ? p.qdst : p.sorted_s)[e];  // (not a copy of m.s: a copy waits for its load)
        const D3 xs = ld3(sorted_X + (int64_t)3 * e);
        m.X[0] = xs.v[0];
        m.X[1] = xs.v[1];
        m.X[2] = xs.v[2];
    };
    // one chunk of n <= 64 markers held one per lane: summed, stored
    auto process_pool = [&](int n, const Mk& m, int am) {
        const bool act = lane < n;
        double acc = 0.0;
        if (act) acc = interp_marker<K>(p, cd, ring, gx0, gy0, zorg, am, m.X, m.s);
        double* dst = (act && m.q >= 0) ? p.Qout + ((int64_t)p.Q_depth * m.q + cd.qcomp) : p.sink + lane;
        *dst = acc;
    };
    double pv[NPT];
    for (int z = a0 + LO + w; z < a0 + HI; z += IWAVES) {
        plane_load(z, pv);
        plane_put(z, pv);
    }
    plane_load(a0 + w + HI, pv);
    GSpan gs;
    gspan_get(a0, gspan_load(a0), gs);
    Mk nxt;
    int anx;
    chunk_load(gs, a0, w, nxt, anx);
    int vsp1 = gspan_load(a0 + IWAVES);
    for (int a = a0; a < a1; a += IWAVES) {
        const int my = a + w;
        lds_barrier();  // the previous group's reads are done
        plane_put(my + HI, pv);
        lds_barrier();  // planes a+LO .. a+IWAVES-1+HI are in the ring
        const Mk cur = nxt;
        const int acur = anx;
        const GSpan gc = gs;

        // prefetch for the next group: its spans (loaded a group ago), its chunk
        // w, the spans of the group after it, plane my+IWAVES+HI
        gspan_get(a + IWAVES, vsp1, gs);
        chunk_load(gs, a + IWAVES, w, nxt, anx);
        vsp1 = gspan_load(a + 2 * IWAVES);
        plane_load(my + IWAVES + HI, pv);
        const int tot = gc.pre[IWAVES];
        if (SW * w < tot) {
            // dense groups: the wave's next chunk loads while this one is summed
            Mk m = cur;
            int am = acur;
            for (int c = w; SW * c < tot; c += IWAVES) {
                const Mk now = m;
                const int anow = am;
                if (SW * (c + IWAVES) < tot) chunk_load(gc, a, c + IWAVES, m, am);
                process_pool(min(tot - SW * c, SW), now, anow);
            }
        }
    }
}

// The three components of an interp item in one workgroup (k_interp3): WPC waves per
// component stage its ring (wave w: component w / WPC; the group's new planes jw, jw + WPC,
// ... of it, jw = w mod WPC), so the workgroup holds three rings (3 x 47 KB for IB_4: one
// workgroup per CU).  The markers are the workgroup's, not a component's: lane L of the
// group takes component L mod 3 of pool marker L / 3 (64 WPC markers a round), so a
// marker's position and index are read once for its three sums -- not once per component
// item -- and the three lanes of a marker store its three Q values next to each other: the
// Q record is written whole, not 8 bytes at a time by three items at three different times.
// Each sum is interp_marker's, in the Fortran order: bitwise the per-component kernel's (and
// the oracle's).  PF groups of planes are in flight per wave in registers (a group's planes
// are loaded PF groups before they are put).  Closed-form kernels, one patch, three
// components.
constexpr int I3C = 3;  // components of a k_interp3 item
// The rings lie RSTR = NSL PVP + I3PAD doubles apart: the three lanes of a marker read the
// same stencil offsets in the three rings, and with rings a multiple of 32 doubles apart
// those reads hit one bank pair (ds_read_b64: a double's banks are its index mod 32) --
// a 3-way conflict on every read (SQ: LDS waits 2.3x the per-component kernel's).  11 and
// 22 doubles apart mod 32 they do not.
constexpr int I3PAD = 11;
// Measured on cfg4 (round 6, profiles/r06): 4 waves a component and one group of planes in
// flight (12 waves, 146 VGPRs) is the fastest form -- 2 waves a component with one or two
// groups in flight 11.7-12.1 ms, 1 wave with two 15.4 ms, components dealt by wave instead
// of by lane 10.4-10.6 ms, against 10.1-10.3 ms -- and still 3-6 % slower than the
// per-component kernel (9.7 ms) although it moves 20 % fewer bytes (44.6 against 55.4 GB
// per launch): one 141-KB workgroup per CU waits at each group's barrier for the slowest
// of its 12 plane loads with nothing else to run, where three independent 4-wave
// workgroups cover each other's waits.  So k_interp_sweep stays the default and this one
// runs on request (ctx_tune interp3 = 1).
constexpr int I3WPC = 4, I3PF = 1;
template <int K> struct I3Sh {
    using S = ISh<K>;
    static constexpr int RSTR = S::NSL * S::PVP + I3PAD;
    static constexpr size_t lds = sizeof(double) * I3C * RSTR;
    static constexpr bool fits = S::FAM == 0 && lds <= 160 * 1024;
};
template <int K, int WPC, int PF>
__global__ __launch_bounds__(SW * I3C * WPC) void k_interp3(Params p) {
    using S = ISh<K>;
    static_assert(I3Sh<K>::fits, "k_interp3: closed-form kernels whose three rings fit the LDS");
    static_assert(IWAVES % WPC == 0, "a component's new planes of a group split evenly over its waves");
    constexpr int LO = S::LO, HI = S::HI, RX = S::RX, NPT = S::NPT, PVP = S::PVP;
    constexpr int PPW = IWAVES / WPC;    // planes a wave stages per group
    constexpr int I3M = WPC * SW;        // pool markers a round
    constexpr int RSTR = I3Sh<K>::RSTR;  // ring stride (doubles)
    __shared__ double ring[I3C * RSTR];
    const int it = sweep_item(p, 1);
    if (it < 0) return;
    const SweepItem si = p.items[it];
    const int col = si.col;
    const int a0 = si.p0, a1 = si.p1;  // the item's anchor planes
    const int lane = lane_id();
    const int w = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
    const int cw = w / WPC, jw = w - cw * WPC;  // the wave's staging: component cw, planes jw + WPC t of a group
    const ColGeom& cg = p.cg;
    const int* const bs = p.plane_start;
    gdouble* const sorted_X = cur_sorted_X(p);
    if (p.zmode) {  // the planes the item reads: a0 + LO .. a1 - 1 + HI
        const bool inner = cg.org[2] + a0 + LO >= p.zlo && cg.org[2] + a1 - 1 + HI <= p.zhi;
        if (inner != (p.zmode == 1)) return;
    }
    {
        bool any = false;  // the same answer in every wave
        for (int a = a0 + lane; a < a1; a += SW) any = any || bs[bucket(cg, a, col, NBAND)] > bs[bucket(cg, a, col, 0)];
        if (!__any(any)) return;
    }
    const int cx = col % cg.ncx, cy = col / cg.ncx;
    const int gx0 = cg.org[0] + cx * COLX + LO, gy0 = cg.org[1] + cy * COLY + LO;
    const int zorg = cg.org[2];
    const int nlast = p.nsorted - 1;
    // ---- staging: the wave's component cw (wave-uniform), as k_interp_sweep stages one
    const CompDesc cd = cw == 0 ? p.comp[0] : (cw == 1 ? p.comp[1] : p.comp[2]);
    auto image = [&](int i, int d) {
        if (!p.iper[d] || (i >= cd.ilower[d] && i <= cd.iupper[d])) return i;
        const int n = cd.iupper[d] - cd.ilower[d] + 1;
        int r = (i - cd.ilower[d]) % n;
        return cd.ilower[d] + (r < 0 ? r + n : r);
    };
    const bool xlast = cd.xcell, ylast = cd.ycell;  // (FAM 0: the unread last staged column / row)
    unsigned poff[NPT];
#pragma unroll
    for (int k = 0; k < NPT; ++k) {
        const int q = min(lane + SW * k, S::PV - 1);
        const int qx = q % RX, qy = q / RX;
        const int gx = gx0 + qx, gy = gy0 + qy;
        const bool in = gx >= cd.lo[0] && gx <= cd.hi[0] && gy >= cd.lo[1] && gy <= cd.hi[1] &&
                        !(xlast && qx == RX - 1) && !(ylast && qy == S::RY - 1);
        poff[k] = in ? 8u * (unsigned)((image(gx, 0) - cd.lo[0]) + (image(gy, 1) - cd.lo[1]) * (int)cd.s1) : OFF_NONE;
    }
    const int plast = a1 - 1 + HI;  // last plane the item reads
    const unsigned plane_bytes = (unsigned)(8 * cd.s2);
    auto plane_load = [&](int zr, double* v) __attribute__((always_inline)) {
        const int z0 = zorg + min(zr, plast);
        const bool zin = z0 >= cd.lo[2] && z0 <= cd.hi[2];
        const int z = zin ? image(z0, 2) : z0;
        const int zc = min(max(z, cd.lo[2]), cd.hi[2]);
        const auto pb = plane_rsrc(cd.u + (int64_t)(zc - cd.lo[2]) * cd.s2, zin ? plane_bytes : 0u);
#pragma unroll
        for (int k = 0; k < NPT; ++k) v[k] = buf_ld(pb, poff[k]);
    };
    double* const ring_w = ring + cw * RSTR;  // the staged component's ring
    auto plane_put = [&](int zr, const double* v) {
        double* sl = ring_w + islot<K>(zr) * PVP;
#pragma unroll
        for (int k = 0; k < NPT; ++k)
            if (S::PV % SW == 0 || k < NPT - 1 || lane + SW * k < S::PV) sl[lane + SW * k] = v[k];
    };
    // ---- the lane's component cl (fixed: 3 I3M lanes a round) and its marker slot
    const int cl = (int)threadIdx.x % I3C, ml = (int)threadIdx.x / I3C;
    CompDesc cdl;
#define I3SEL(f) cdl.f = cl == 0 ? p.comp[0].f : (cl == 1 ? p.comp[1].f : p.comp[2].f)
#pragma unroll
    for (int d = 0; d < 3; ++d) {
        I3SEL(xlo[d]);
        I3SEL(ilower[d]);
        I3SEL(lo[d]);
        I3SEL(hi[d]);
    }
    I3SEL(axis);
    I3SEL(xcell);
    I3SEL(ycell);
    I3SEL(qcomp);
#undef I3SEL
    const double* const ring_l = ring + cl * RSTR;
    struct Mk {
        int q;  // the marker whose Q this entry writes (-1: a later duplicate entry does)
        double X[3];
    };
    auto lds_barrier = [&]() {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
    };
    struct GSpan {
        int beg[IWAVES];
        int pre[IWAVES + 1];
    };
    auto gspan_load = [&](int a) {
        const int k = lane < IWAVES ? lane : min(lane - IWAVES, IWAVES - 1);
        const int ac = min(a + k, cg.nz - 1);
        return bs[bucket(cg, ac, col, lane >= IWAVES && lane < 2 * IWAVES ? NBAND : 0)];
    };
    auto gspan_get = [&](int a, int v, GSpan& gsp) {
        int acc = 0;
#pragma unroll
        for (int k = 0; k < IWAVES; ++k) {
            const int b = __builtin_amdgcn_readlane(v, k);
            const int e = a + k < a1 ? __builtin_amdgcn_readlane(v, IWAVES + k) : b;
            gsp.beg[k] = b;
            gsp.pre[k] = acc;
            acc += e - b;
        }
        gsp.pre[IWAVES] = acc;
    };
    // round r of a group: pool marker I3M r + ml (clamped), with its anchor plane
    auto mk_load = [&](const GSpan& gsp, int a, int r, Mk& m, int& am) {
        const int tot = gsp.pre[IWAVES];
        const int j = min(I3M * r + ml, max(tot - 1, 0));
        int e = gsp.beg[0] + j, k = 0;
#pragma unroll
        for (int q = 1; q < IWAVES; ++q)
            if (j >= gsp.pre[q]) {
                e = gsp.beg[q] + (j - gsp.pre[q]);
                k = q;
            }
        am = a + k;
        e = min(e, nlast);
        m.q = (p.qdst ? p.qdst : p.sorted_s)[e];
        const D3 xs = ld3(sorted_X + (int64_t)3 * e);
        m.X[0] = xs.v[0];
        m.X[1] = xs.v[1];
        m.X[2] = xs.v[2];
    };
    auto process = [&](int n, const Mk& m, int am) {  // round of n <= I3M markers
        const bool act = ml < n;
        double acc = 0.0;
        if (act) acc = interp_marker<K>(p, cdl, ring_l, gx0, gy0, zorg, am, m.X, 0);
        double* dst = (act && m.q >= 0) ? p.Qout + ((int64_t)p.Q_depth * m.q + cdl.qcomp) : p.sink + lane;
        *dst = acc;
    };
    {  // prologue: planes a0 + LO .. a0 + HI - 1 into the rings
        double pv[NPT];
        for (int z = a0 + LO + jw; z < a0 + HI; z += WPC) {
            plane_load(z, pv);
            plane_put(z, pv);
        }
    }
    // pv[b][t]: the group's new plane jw + WPC t, in register buffer b (b = group index mod PF)
    double pv[PF][PPW][NPT];
#pragma unroll
    for (int b = 0; b < PF; ++b)
#pragma unroll
        for (int t = 0; t < PPW; ++t) plane_load(a0 + b * IWAVES + jw + WPC * t + HI, pv[b][t]);
    GSpan gs;
    gspan_get(a0, gspan_load(a0), gs);
    Mk nxt;
    int anx;
    mk_load(gs, a0, 0, nxt, anx);
    int vsp1 = gspan_load(a0 + IWAVES);
    auto group = [&](int a, double (*pvb)[NPT]) __attribute__((always_inline)) {
        lds_barrier();  // the previous group's reads are done
#pragma unroll
        for (int t = 0; t < PPW; ++t) plane_put(a + jw + WPC * t + HI, pvb[t]);
        lds_barrier();  // planes a+LO .. a+IWAVES-1+HI of every component are in the rings
        const Mk cur = nxt;
        const int acur = anx;
        const GSpan gc = gs;
        gspan_get(a + IWAVES, vsp1, gs);
        mk_load(gs, a + IWAVES, 0, nxt, anx);
        vsp1 = gspan_load(a + 2 * IWAVES);
#pragma unroll
        for (int t = 0; t < PPW; ++t) plane_load(a + PF * IWAVES + jw + WPC * t + HI, pvb[t]);
        const int tot = gc.pre[IWAVES];
        Mk m = cur;
        int am = acur;
        for (int r = 0; I3M * r < tot; ++r) {  // (dense groups: the next round loads while this one sums)
            const Mk now = m;
            const int anow = am;
            if (I3M * (r + 1) < tot) mk_load(gc, a, r + 1, m, am);
            process(min(tot - I3M * r, I3M), now, anow);
        }
    };
    for (int a = a0; a < a1; a += PF * IWAVES) {
#pragma unroll
        for (int b = 0; b < PF; ++b)
            if (b == 0 || a + b * IWAVES < a1) group(a + b * IWAVES, pv[b]);
    }
}

// Entries binned "outside" (no stencil point can reach any array): V = 0.
__global__ __launch_bounds__(BLOCK) void k_interp_outside_col(Params p, int n) {
    const int first = p.plane_start[p.nbuckets_total];
    for (int e = first + blockIdx.x * BLOCK + threadIdx.x; e < n; e += gridDim.x * BLOCK) {
        const int s = p.qdst ? p.qdst[e] : p.sorted_s[e];
        if (s < 0) continue;
        for (int c = 0; c < p.ncomp; ++c) p.Qout[(int64_t)p.Q_depth * s + p.comp[c].qcomp] = 0.0;
    }
}

// ---------------------------------------------------------------------------
// spreading
// ---------------------------------------------------------------------------
// The ring holds one plane of the column's 32 x COLY owned points per slot, in
// 4 x 4 tiles of 16 consecutive doubles: point (x, y) at
//     16 ((x >> 2) + (COLX / 4) (y >> 2)) + (x & 3) + 4 (y & 3).
// ds_add_f64 serves a wave as 4 groups of 16 lanes, each conflict-free when its
// f64 indices differ mod 16 (tools/ubench_lds2.hip; the microarchitecture
// guide's ds_write_b64 row), and a point's index mod 16 -- its bank class -- is
// (x & 3) + 4 (y & 3) in every tile of every slot.  The 4 x 4 points (i0, i1) of
// a 4-wide stencil plane therefore cover the 16 classes once each, whatever the
// stencil's position, and the lanes can take them in an order in which the 16
// lanes of a group always hit 16 different classes (spread_tiled).
// ZC: the component's z frame is the bin keys' (cell) frame, where the closed-form
// kernels' (FAM 0) stencil planes of anchor a are exactly a + [LO, HI - 1]
// (ic_lower = NINT - W/2): the ring is one slot shorter (IB_4: 5 slots, 20 KB,
// 8 waves per CU instead of 6).
template <int K, bool ZC = false> struct SSh {
    using T = KT<K>;
    static constexpr int W = T::W, LO = T::LO, HI = T::HI, FAM = T::FAM;
    static_assert(!ZC || FAM == 0, "the key-frame ring: closed-form kernels");
    static constexpr int HIE = ZC ? HI - 1 : HI;  // highest plane an anchor reaches (relative)
    static constexpr int NS = HIE - LO + 1;       // planes an anchor plane reaches
    static constexpr int NSL = NS + 1;            // ring slots: the planes two anchors reach
    static constexpr int PV = COLX * COLY;   // owned points per plane = doubles per slot
    static constexpr int NPL = PV / SW;      // staged points per lane and plane
    static constexpr int NR = 11;            // candidate ranges per anchor plane
    static_assert(NS <= 16, "plane field");
    static_assert(COLX == 32 && COLY % 4 == 0 && COLY >= 8, "32-point rows of 4 x 4 tiles; bands need COLY >= 8");
};

// (x, y) in the column of the tile-major slot index i
__device__ __forceinline__ void ring_xy(int i, int& x, int& y) {
    const int t = i >> 4, j = i & 15;
    x = 4 * (t % (COLX / 4)) + (j & 3);
    y = 4 * (t / (COLX / 4)) + (j >> 2);
}
// slot index of (x, y), both wrapped into the column (x mod 32, y mod COLY keep
// the bank class: 32 and COLY are multiples of 4)
__device__ __forceinline__ int ring_wrapped(int x, int y) {
    const int xw = x & (COLX - 1);
    const int yw = ((y % COLY) + COLY) % COLY;
    return 16 * ((xw >> 2) + (COLX / 4) * (yw >> 2)) + (xw & 3) + 4 * (yw & 3);
}

template <class S> __device__ __forceinline__ int sslot(int prel) {
    return (int)((unsigned)(prel + 16 * S::NSL) % (unsigned)S::NSL);  // prel >= -HI + LO > -16*NSL
}

// The candidate ranges of anchor plane a for column (cx, cy), in sorted (bucket)
// order, from the bucket-start table row t[r][i] = bs(a, col(cx-1, cy-1+r), 0) + i
// (i < 28: bands of columns cx-1, cx, cx+1).  Row cy-1 (south): the markers
// reaching north (yb = 2); row cy: those reaching the column (west: xb = 2, own:
// all, east: xb = 0 -- one contiguous range); row cy+1: those reaching south.
struct Ranges {
    int start[SSh<K_IB_4>::NR];
    int pre[SSh<K_IB_4>::NR + 1];
};
// rows held one entry per lane (lane k: entry k of the row): wave-uniform reads
__device__ __forceinline__ void make_ranges_lanes(const int* rowv, Ranges& R) {
    constexpr int NR = SSh<K_IB_4>::NR;
    constexpr int rr[NR] = {0, 0, 0, 0, 0, 1, 2, 2, 2, 2, 2};
    constexpr int ib[NR] = {8, 11, 14, 17, 20, 6, 6, 9, 12, 15, 18};
    constexpr int ie[NR] = {9, 12, 15, 18, 21, 21, 7, 10, 13, 16, 19};
    int acc = 0;
#pragma unroll
    for (int r = 0; r < NR; ++r) {
        const int b = __builtin_amdgcn_readlane(rowv[rr[r]], ib[r]);
        const int e = __builtin_amdgcn_readlane(rowv[rr[r]], ie[r]);
        R.start[r] = b;
        R.pre[r] = acc;
        acc += e - b;
    }
    R.pre[NR] = acc;
}
// sorted position of candidate j (< pre[NR])
__device__ __forceinline__ int range_pos(const Ranges& R, int j) {
    constexpr int NR = SSh<K_IB_4>::NR;
    int pos = R.start[0] + j;
#pragma unroll
    for (int r = 1; r < NR; ++r)
        if (j >= R.pre[r]) pos = R.start[r] + (j - R.pre[r]);
    return pos;
}

// ---------------------------------------------------------------------------
// the spread's candidate stream (built once per binning, on the first spread)
// ---------------------------------------------------------------------------
// Per (patch, column, anchor plane) -- "column-anchor" ca, column-major within a
// patch (ca = bucket_base / NBAND + col * nz + a) -- the sorted positions of the
// markers whose stencil reaches the column from that anchor plane: the 11 ranges of
// make_ranges_lanes, in that order.  A column's anchors are consecutive, so chunk 1
// of an anchor (the previous anchor's leftovers, then its own first) is one piece of
// the stream, and the sweep needs no range arithmetic per chunk.  k_cand_count: the
// lengths; an exclusive scan: cs_off; k_cand_write: the positions (a wave per ca).
// The shifted-z frame (closed-form kernels, cs_off_z set).  A component whose z frame is
// shifted by -dz/2 (side-z, node and x/y-edge data) has its stencil planes at a' + [LO,
// HI - 1] for its own anchor a' = NINT in that frame (ic_lower = NINT - W/2), and a' is
// the key anchor a or a + 1.  k_cand_write puts each anchor's candidates with a' = a
// first (in range order) and those with a' = a + 1 after them (in reverse range order),
// so the candidates of shifted anchor a' -- the upper ones of a' - 1, then the lower ones
// of a' -- are again one piece of the stream, [cs_off_z[zb], cs_off_z[zb + 1]) with zb =
// ca_base_z + col (nz + 1) + a' (a' = 0 .. nz): such a component's ring needs the
// key-frame components' slots (5 for IB_4), not one more.
// (zb: the column-anchor's index in the shifted-z frame, patch base ca_base_z + col (nz + 1)
// + a; zxlo, zilo: the z origin of that frame, x_lower - dz / 2, and the z ilower.  ptab:
// the patches' first column-anchors in LDS (cs_patch_table), else searched in p.pd)
constexpr int CS_PTAB = 2048;
__device__ __forceinline__ bool ca_decode(const Params& p, int ca, ColGeom& cg, int& col, int& a, const int*& bs,
                                          int& zb, double& zxlo, int& zilo, const int* ptab) {
    int base = 0;
    if (p.pd) {
        int lo = 0, hi = p.npatch - 1;
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if ((ptab ? ptab[mid] : p.pd[mid].bucket_base / NBAND) <= ca) lo = mid;
            else hi = mid - 1;
        }
        const PatchDesc& P = p.pd[lo];
        cg = P.cg;
        base = P.bucket_base / NBAND;
        bs = p.plane_start + P.bucket_base;
        zb = P.ca_base_z;
        zxlo = P.xlo[2] - 0.5 * p.bg.dx[2];  // (make_comps' frame shift)
        zilo = P.ilower[2];
    } else {
        cg = p.cg;
        bs = p.plane_start;
        zb = 0;
        zxlo = p.bg.xlo[2] - 0.5 * p.bg.dx[2];
        zilo = p.bg.ilower[2];
    }
    const int l = ca - base;
    col = l / cg.nz;
    a = l - col * cg.nz;
    zb += col * (cg.nz + 1) + a;
    const int cx = col % cg.ncx, cy = col / cg.ncx;
    return !(cx == 0 || cx == cg.ncx - 1 || cy == 0 || cy == cg.ncy - 1);  // guard columns: no items
}
// the 11 candidate ranges of (column col, anchor a): begin / end sorted positions
__device__ __forceinline__ void ca_range(const ColGeom& cg, const int* bs, int col, int a, int r, int& b, int& e) {
    constexpr int rr[11] = {0, 0, 0, 0, 0, 1, 2, 2, 2, 2, 2};
    constexpr int ib[11] = {8, 11, 14, 17, 20, 6, 6, 9, 12, 15, 18};
    constexpr int ie[11] = {9, 12, 15, 18, 21, 21, 7, 10, 13, 16, 19};
    const int cx = col % cg.ncx, cy = col / cg.ncx;
    const int base = bucket(cg, a, (cy - 1 + rr[r]) * cg.ncx + (cx - 1), 0);
    b = bs[base + ib[r]];
    e = bs[base + ie[r]];
}
// (grid-stride loops over the column-anchors on a bounded grid: with nothing moved
// the launches return at once, and cfg5's 0.5 M column-anchors, mostly empty, cost
// no launch of their own)
constexpr int CS_GRID = 8192;
// a re-binning that moved nothing (and, for a split stream, changed no shifted-z anchor):
// the stream stands
__device__ __forceinline__ bool cs_stands(const Params& p) {
    return p.items_skip && *p.items_skip == 0 && (!p.cs_off_z || *p.cs_zflip != p.cs_epoch);
}
// a level's patch search in LDS: the first column-anchor of every patch (a dependent chain
// of ~9 loads from the patch table per column-anchor otherwise; cfg5 has 0.8 M of them)
__device__ __forceinline__ const int* cs_patch_table(const Params& p, int* ptab) {
    if (!p.pd || p.npatch > CS_PTAB) return nullptr;
    for (int q = threadIdx.x; q < p.npatch; q += BLOCK) ptab[q] = p.pd[q].bucket_base / NBAND;
    __syncthreads();
    return ptab;
}
__global__ __launch_bounds__(BLOCK) void k_cand_count(Params p, int ncl, int* cnt) {
    if (cs_stands(p)) return;
    __shared__ int ptab_s[CS_PTAB];
    const int* const ptab = cs_patch_table(p, ptab_s);
    for (int ca = blockIdx.x * BLOCK + threadIdx.x; ca < ncl; ca += gridDim.x * BLOCK) {
        ColGeom cg;
        int col, a, zb, zilo;
        double zxlo;
        const int* bs;
        int t = 0;
        if (ca_decode(p, ca, cg, col, a, bs, zb, zxlo, zilo, ptab)) {
#pragma unroll
            for (int r = 0; r < 11; ++r) {
                int b, e;
                ca_range(cg, bs, col, a, r, b, e);
                t += e - b;
            }
        }
        cnt[ca] = t;
    }
}
// a wave per column-anchor: its three rows of bucket starts one entry a lane (three
// coalesced loads), the ranges made once (make_ranges_lanes), then stream entry j of it
// by range_pos, 64 a store.  SHZ: split by the shifted anchor (a ballot compaction from
// each end) and the shifted-z boundary cs_off_z[zb + 1] written; lane 0 of the wave that
// takes a column's anchor 0 writes its column's first boundary, cs_off_z[zb] = cs_off[ca].
// The candidates' loads are unconditional (indices clamped), so that no branch waits on
// them; on a level an empty column-anchor skips its rows (one wait on its two offsets).  (Two
// column-anchors a pass, their loads issued together, measured 0.1-0.15 ms slower on cfg4
// and cfg5 --move, profiles/r05x.)
struct CaJob {
    ColGeom cg;
    int col, a, zb, zilo, o, t;
    double zxlo;
    bool items;
    const int* bs;
    int rowv[3];
    Ranges R;
    int e0;     // the lane's first candidate (clamped into the stream piece)
    double z0;  // its z (SHZ)
};
template <bool SHZ>
__global__ __launch_bounds__(BLOCK) void k_cand_write(Params p, int ncl, const int* off, int* pos,
                                                      const unsigned long long* total) {
    if (cs_stands(p)) return;
    // a stream of 2^31 entries or more: its 32-bit offsets wrapped; nothing is written and
    // device flag 16 says so at the next synchronize (the sweeps' reads stay clamped)
    if (*total >= (unsigned long long)p.cs_total + 1ull) {
        if (blockIdx.x == 0 && threadIdx.x == 0) atomicOr(p.err, 16);
        return;
    }
    const int lane = threadIdx.x & (SW - 1);
    const int nw = gridDim.x * (BLOCK / SW);
    gdouble* const sX = cur_sorted_X(p);
    const double inv_dz = 1.0 / p.bg.dx[2];
    int* const offz = const_cast<int*>(p.cs_off_z);
    __shared__ int ptab_s[CS_PTAB];
    const int* const ptab = cs_patch_table(p, ptab_s);
    auto load_rows = [&](int ca, CaJob& J) {
        J.items = ca < ncl && ca_decode(p, ca, J.cg, J.col, J.a, J.bs, J.zb, J.zxlo, J.zilo, ptab);
        J.o = off[min(ca, ncl - 1)];
        // on a level an empty column-anchor (most of a clustered level's) loads no rows; one
        // patch of uniform markers has few, and would only wait for the offsets
        if (p.pd) J.items = J.items && off[min(ca + 1, ncl)] != J.o;
        if (J.items) {
            const int cx = J.col % J.cg.ncx, cy = J.col / J.cg.ncx;
            const int col0 = (cy - 1) * J.cg.ncx + (cx - 1);
#pragma unroll
            for (int r = 0; r < 3; ++r) J.rowv[r] = J.bs[bucket(J.cg, J.a, col0 + r * J.cg.ncx, 0) + min(lane, 27)];
        }
    };
    auto load_first = [&](CaJob& J) {
        J.t = 0;
        J.e0 = 0;
        J.z0 = 0.0;
        if (!J.items) return;
        make_ranges_lanes(J.rowv, J.R);
        J.t = J.R.pre[SSh<K_IB_4>::NR];
        J.e0 = range_pos(J.R, min(lane, max(J.t - 1, 0)));
        if constexpr (SHZ) J.z0 = sX[(int64_t)3 * min(J.e0, p.nsorted - 1) + 2];  // (t = 0: e0 may be n)
    };
    auto finish = [&](int ca, CaJob& J) {
        if (ca >= ncl) return;
        const int o = J.o;
        if (SHZ && lane == 0) {
            if (J.a == 0) offz[J.zb] = o;
            if (ca == ncl - 1) offz[J.zb + 2] = off[ca + 1];  // the stream's end (a' = nz + 1 of the last column)
        }
        const int t = J.t;
        if constexpr (!SHZ) {
            if (lane < t) pos[o + lane] = J.e0;
            for (int j = lane + SW; j < t; j += SW) pos[o + j] = range_pos(J.R, j);
        } else {
            const int aa = J.a + J.cg.org[2] - J.zilo;  // the key anchor as a shifted-frame NINT
            int nlo = 0, nup = 0;
            for (int j0 = 0; j0 < t; j0 += SW) {
                const int j = j0 + lane;
                int e = J.e0;
                double z = J.z0;
                if (j0 > 0) {
                    e = range_pos(J.R, min(j, t - 1));
                    z = sX[(int64_t)3 * e + 2];
                }
                const double xo = (z - J.zxlo) * inv_dz;
                const int n = p.cs_rint ? (int)__builtin_rint(xo) : d_nint(xo);
                const bool in = j < t;
                const bool up = in && n > aa;  // n = aa + 1 (the binning invariant: aa or aa + 1)
                const unsigned long long bu = __ballot(up), bl = __ballot(in && !up);
                const unsigned long long below = (1ull << lane) - 1ull;
                if (in) {
                    if (up) pos[o + t - 1 - (nup + __popcll(bu & below))] = e;
                    else pos[o + nlo + __popcll(bl & below)] = e;
                }
                nlo += __popcll(bl);
                nup += __popcll(bu);
            }
            if (lane == 0) offz[J.zb + 1] = o + nlo;
        }
    };
    for (int ca = blockIdx.x * (BLOCK / SW) + (int)(threadIdx.x / SW); ca < ncl; ca += nw) {
        CaJob J;
        load_rows(ca, J);
        load_first(J);
        finish(ca, J);
    }
}
hipError_t launch_cand_stream(const Params& p, int ncl, int* cnt, int* off, int* pos, void* temp, size_t temp_bytes,
                              unsigned long long* total, hipStream_t s) {
    if (ncl <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_cand_count, dim3(std::min((ncl + BLOCK - 1) / BLOCK, CS_GRID)), dim3(BLOCK), 0, s, p, ncl,
                       cnt);
    // the stream's length in 64 bits beside the 32-bit scan (k_cand_write checks it), where
    // it could reach 2^31 (the 4-a-marker bound, p.cs_total, is 2^31 - 1); else 0
    hipError_t e = hipMemsetAsync(total, 0, sizeof(unsigned long long), s);
    if (e != hipSuccess) return e;
    if (p.cs_total >= 0x7fffffff && (e = launch_sum64(cnt, ncl, total, s)) != hipSuccess) return e;
    e = launch_scan(temp, temp_bytes, cnt, off, ncl + 1, s);  // cnt[ncl] = 0: off[ncl] = the total
    if (e != hipSuccess) return e;
    const int per = BLOCK / SW;
    const dim3 g(std::min((ncl + per - 1) / per, CS_GRID)), b(BLOCK);
    if (p.cs_off_z) hipLaunchKernelGGL(k_cand_write<true>, g, b, 0, s, p, ncl, off, pos, total);
    else hipLaunchKernelGGL(k_cand_write<false>, g, b, 0, s, p, ncl, off, pos, total);
    return hipGetLastError();
}

// candidate data of one lane
struct Cand {
    double X[3];
    double V;
    int s;
};

// w[s] <- w[(s + r) & 3] for s < 4 (a two-stage barrel of selects)
template <typename T> __device__ __forceinline__ void rot4(T* w, int r) {
    const bool b0 = r & 1, b1 = r & 2;
    const T c0 = b0 ? w[1] : w[0], c1 = b0 ? w[2] : w[1], c2 = b0 ? w[3] : w[2], c3 = b0 ? w[0] : w[3];
    w[0] = b1 ? c2 : c0;
    w[1] = b1 ? c3 : c1;
    w[2] = b1 ? c0 : c2;
    w[3] = b1 ? c1 : c3;
}

// The adds of one staged candidate per lane: the lane computes its three 1-D
// stencils, then issues its W^3 adds as ds_add_f64, plane by plane.
// Conflict-free order: lane l = 16 g + 4 jy + jx takes, at step (s0, s1) of a
// stencil plane (s0, s1 < 4), its point whose x = s0 + jx and y = s1 + jy
// (mod 4) -- a rotation of its stencil's first four columns and rows by
// (jx - ox) and (jy - oy) mod 4 -- so the 16 lanes of every lane group hit the
// 16 bank classes once each, in every instruction, wherever the stencils lie
// (no ranking or dealing of the candidates).  IB_6 adds its 6 x 6 plane in 40
// steps (tiled6): the rotated 4 x 4 first, then a second rotated round in which
// the step of relative class (cx, cy) takes the point (cx + 4, cy) for cx < 2,
// (cx, cy + 4) for cx >= 2 > cy, and a weight-0 add for cx, cy >= 2 -- conflict-free
// as the first, since a stencil column cx + 4 has the bank class of column cx --
// and last the 8 points of rows 4, 5 and columns {0, 1, 4, 5}, whose classes
// repeat (so 8 of 40 adds can conflict, against 20 of 36 unrotated).  IB_4_W8
// turns each of its four 4 x 4 blocks alike (all 64 conflict-free); narrower
// stencils go unrotated.
// A stencil point that is clipped (outside the ghost box) or not owned (outside
// the column, or in a neighbour item's planes) is added with weight 0 at its
// position wrapped into the column (a +0 on an owned point of the same class),
// so a plane's adds need no per-point branch; whole planes that are clipped or
// not owned are skipped with one exec mask each.  Adding +-0 changes no value,
// except that a -0.0 it lands on becomes +0.0.  Within one instruction the
// lanes that hit the same point add in lane order, so every point receives its
// contributions in a fixed order (bit-stable).
// `before` runs on every lane after the weights are computed and before any add
// (the anchor step's writeback stores go there: issued after the candidate loads
// they would otherwise be counted ahead of, and while the previous adds drain).
// The work is split in two: spread_setup (the stencils, weights and offsets, into
// a TileAdds) and spread_adds (the ring adds), so that a dense anchor's full
// chunks can be set up two at a time before either's adds (k_spread_sweep).
template <int W> struct TileAdds {
    static constexpr int NA = W == 6 ? 40 : W * W;  // adds per stencil plane
    double P[NA];  // products of the x and y weights, in issue order
    int off[NA];   // their points' byte offsets in a slot
    double wz[W];
    int z0, z1;    // the stencil planes added (none: z0 > z1)
    int sl;        // ring slot of stencil plane 0
};
template <int K, bool CNT, bool ZC, typename Before>
__device__ __forceinline__ void spread_setup(const Params& p, const CompDesc& cd, const Cand& cdat, bool act, int a,
                                             int X0, int Y0, int zorg, int xlo, int xhi, int ylo, int yhi, int plo,
                                             int phi, double inv_h3, const double* inv_d, unsigned long long* cnt,
                                             Before&& before, TileAdds<SSh<K, ZC>::W>& T) {
    using S = SSh<K, ZC>;
    constexpr int W = S::W, FAM = S::FAM, NSL = S::NSL;
    constexpr bool ROT = W >= 4;
    St<W> st[3];
#pragma unroll
    for (int d = 0; d < 3; ++d) {
        const double Xraw = (FAM == 2) ? p.X[(int64_t)3 * cdat.s + d] : cdat.X[d];
        // X/dx by a multiply (see stencil1d for ties)
#if IBTK_LE_DIAG_SPREAD & 2  // diagnostic: trivial weights (results wrong by design)
        {
            const double xo = (cdat.X[d] - cd.xlo[d]) * inv_d[d];
            st[d].icl = (int)__builtin_rint(xo) + cd.ilower[d] - W / 2;
            st[d].ist = 0;
            st[d].isp = W - 1;
#pragma unroll
            for (int i = 0; i < W; ++i) st[d].w[i] = 0.25 + 0.01 * i;
            (void)Xraw;
        }
#else
        if constexpr (K == K_IB_4) {
            // IB_4 (f.m4:1447-1457) with X/dx by a multiply and the anchor by rint: NINT
            // differs from it only at a tie, where the stencil one cell over carries the
            // same weights on the same points (the end weight is 0 at r = 0 or 1).  The
            // weights keep 0.125 (a -+ q) unscaled here (t[]): the x / z scalings below
            // fold 0.125 into V / 1 / h^3 -- exact powers of two, the same bits.
            const double xo = (cdat.X[d] - cd.xlo[d]) * inv_d[d];
            const double n = __builtin_rint(xo);
            st[d].icl = (int)n + cd.ilower[d] - 2;
            const double r = xo - (n - 0.5);
            const double q = sqrt_1_2(1.0 + 4.0 * r * (1.0 - r));
            const double ta = 3.0 - 2.0 * r, tb = 1.0 + 2.0 * r;
            st[d].w[0] = ta - q;
            st[d].w[1] = ta + q;
            st[d].w[2] = tb + q;
            st[d].w[3] = tb - q;
            st[d].ist = max(cd.lo[d] - st[d].icl, 0);
            st[d].isp = 3 - max(st[d].icl + 3 - cd.hi[d], 0);
            (void)Xraw;
        } else {
            stencil1d<K, true>(cdat.X[d], Xraw, cd.xlo[d], p.bg.dx[d], cd.ilower[d], cd.lo[d], cd.hi[d],
                               d == cd.axis, p.K6, st[d], inv_d[d]);
        }
#endif
    }
    // IB_4: the weights above are 8 w; 0.125 goes into the x and z scalings (exact)
    const double sx = K == K_IB_4 ? 0.125 * cdat.V : cdat.V;
    const double sy = K == K_IB_4 ? 0.125 : 1.0;
    const double sz = K == K_IB_4 ? 0.125 * inv_h3 : inv_h3;
    const int ox = st[0].icl - X0, oy = st[1].icl - Y0, oz = st[2].icl - (zorg + a);
    // binning invariant: every stencil index lies in [key + LO, key + HI] and the
    // candidates' key cells lie within HI / -LO of the column (key_band), +-1 for
    // a NINT tie of the multiply.  The ring addresses are wrapped, so memory
    // stays safe anyway.
    constexpr int LO = S::LO, HI = S::HI;
    const bool bad = ox < LO - HI - 1 || ox + W - 1 > COLX - LO + HI || oy < LO - HI - 1 || oy + W - 1 > COLY - LO + HI;
    if (act && bad) atomicOr(p.err, 2);
    before();
    const bool go = act && !bad;  // idle lanes sit the adds out (no planes)
    // owned and clipped-in ranges of the stencil indices
    const int x0 = max(st[0].ist, xlo - ox), x1 = min(st[0].isp, xhi - ox);
    const int y0 = max(st[1].ist, ylo - oy), y1 = min(st[1].isp, yhi - oy);
    // planes within the ring's reach of the lane's anchor, [LO, HIE] (a stencil
    // moved by a NINT tie of the multiply -- a weight of an ulp's order -- is cut there)
    T.z0 = go ? max(max(st[2].ist, plo - (a + oz)), S::LO - oz) : W;
    T.z1 = min(min(st[2].isp, phi - (a + oz)), S::HIE - oz);
    T.sl = (int)((unsigned)(a + oz + 64 * NSL) % (unsigned)NSL);
    double wx[W], wy[W];
    double* const wz = T.wz;
#pragma unroll
    for (int i = 0; i < W; ++i) {
        wx[i] = (i >= x0 && i <= x1) ? st[0].w[i] * sx : 0.0;  // V applied first (f.m4:1512-1513 up to rounding)
        wy[i] = (i >= y0 && i <= y1) ? (K == K_IB_4 ? st[1].w[i] * sy : st[1].w[i]) : 0.0;
        wz[i] = st[2].w[i] * sz;  // planes outside [z0, z1] are skipped below
    }
    // byte offsets in a slot of stencil column / row s: the x and y parts of
    // ring_wrapped
    auto xpart = [&](int s) {
        const int xw = (ox + s) & (COLX - 1);
        return 8 * (16 * (xw >> 2) + (xw & 3));
    };
    auto ypart = [&](int s) {
        const int yw = (((oy + s) % COLY) + COLY) % COLY;
        return 8 * (16 * (COLX / 4) * (yw >> 2) + 4 * (yw & 3));
    };
    // the plane's adds: products of the x and y weights and the byte offsets of
    // their points in a slot, in issue order
    constexpr int NA = TileAdds<W>::NA;
    int* const off = T.off;
    double* const P = T.P;
    if constexpr (W == 6) {  // tiled6 (see above)
        const int lane = lane_id();
        const int jx = lane & 3, jy = (lane >> 2) & 3;
        const int rx = (jx - ox) & 3, ry = (jy - oy) & 3;
        int bxa[6], bya[6];
#pragma unroll
        for (int s = 0; s < 6; ++s) {
            bxa[s] = xpart(s);
            bya[s] = ypart(s);
        }
        // round 3: columns {0, 1, 4, 5} turned by jx, rows {4, 5} by jy (a partial spread)
        double x3[4] = {wx[0], wx[1], wx[4], wx[5]};
        int bx3[4] = {bxa[0], bxa[1], bxa[4], bxa[5]};
        rot4(x3, jx);
        rot4(bx3, jx);
        const bool sy = jy & 1;
        const double y3[2] = {sy ? wy[5] : wy[4], sy ? wy[4] : wy[5]};
        const int by3[2] = {sy ? bya[5] : bya[4], sy ? bya[4] : bya[5]};
        // rounds 1 and 2: entry s of a rotated vector is relative class (s + r) & 3
        double x4[4] = {wx[4], wx[5], 0.0, 0.0}, y4[4] = {wy[4], wy[5], 0.0, 0.0};
        int bx4[4] = {bxa[4], bxa[5], bxa[2], bxa[3]}, by4[4] = {bya[4], bya[5], bya[2], bya[3]};
        int bxr[4] = {bxa[0], bxa[1], bxa[2], bxa[3]}, byr[4] = {bya[0], bya[1], bya[2], bya[3]};
        rot4(wx, rx);
        rot4(x4, rx);
        rot4(bx4, rx);
        rot4(bxr, rx);
        rot4(wy, ry);
        rot4(y4, ry);
        rot4(by4, ry);
        rot4(byr, ry);
#pragma unroll
        for (int s1 = 0; s1 < 4; ++s1)
#pragma unroll
            for (int s0 = 0; s0 < 4; ++s0) {
                const int k = 4 * s1 + s0;
                P[k] = wx[s0] * wy[s1];
                off[k] = bxr[s0] + byr[s1];
                const bool lo = ((s0 + rx) & 3) < 2;  // cx < 2: column cx + 4, row cy
                P[16 + k] = lo ? x4[s0] * wy[s1] : wx[s0] * y4[s1];
                off[16 + k] = lo ? bx4[s0] + byr[s1] : bxr[s0] + by4[s1];
            }
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                P[32 + 4 * u + t] = x3[t] * y3[u];
                off[32 + 4 * u + t] = bx3[t] + by3[u];
            }
    } else {
        static_assert(!ROT || W % 4 == 0, "rotated blocks of 4");
        int rx = 0, ry = 0;
        if constexpr (ROT) {
            const int lane = lane_id();
            rx = ((lane & 3) - ox) & 3;
            ry = (((lane >> 2) & 3) - oy) & 3;
            // every aligned block of 4 columns (rows) turned alike: stencil column
            // 4 i + c has the bank class of column c (IB_4_W8: 64 steps, all conflict-free)
#pragma unroll
            for (int b = 0; b + 4 <= W; b += 4) {
                rot4(wx + b, rx);
                rot4(wy + b, ry);
            }
        }
        int bx[W], by[W];
        if constexpr (ROT && COLY == 16) {
            // Step s of a block of 4 takes the stencil column x = ox + c, c = (s + rx) & 3,
            // whose x & 3 is cls = (s + lane) & 3 (a lane constant) and whose x >> 2 is
            // (ox >> 2) + [cls < (ox & 3)]: its offset in a slot, 128 ((x >> 2) & 7) + 8 cls,
            // needs a compare and a select per step (likewise the rows, 1024 ((y >> 2) & 3) + 32 cls)
            const int lane = lane_id();
            const int qx = ox >> 2, rxl = ox & 3, qy = oy >> 2, ryl = oy & 3;
#pragma unroll
            for (int b = 0; b < W; b += 4) {
                const int hx0 = 128 * ((qx + b / 4) & 7), hx1 = 128 * ((qx + b / 4 + 1) & 7);
                const int hy0 = 1024 * ((qy + b / 4) & 3), hy1 = 1024 * ((qy + b / 4 + 1) & 3);
#pragma unroll
                for (int s = 0; s < 4; ++s) {
                    const int cx = (s + lane) & 3, cy = (s + (lane >> 2)) & 3;
                    bx[b + s] = (cx < rxl ? hx1 : hx0) | (8 * cx);
                    by[b + s] = (cy < ryl ? hy1 : hy0) | (32 * cy);
                }
            }
        } else {
#pragma unroll
            for (int s = 0; s < W; ++s) {
                bx[s] = xpart(ROT ? (s & ~3) + (((s & 3) + rx) & 3) : s);
                by[s] = ypart(ROT ? (s & ~3) + (((s & 3) + ry) & 3) : s);
            }
        }
#pragma unroll
        for (int s1 = 0; s1 < W; ++s1)
#pragma unroll
            for (int s0 = 0; s0 < W; ++s0) {
                off[s1 * W + s0] = bx[s0] + by[s1];
                P[s1 * W + s0] = wx[s0] * wy[s1];
            }
    }
    if constexpr (CNT) {  // counted launch (ibtk_le_ctx_count_adds): the adds issued below
#pragma unroll
        for (int i2 = 0; i2 < W; ++i2) {
            const unsigned long long bm = __ballot(i2 >= T.z0 && i2 <= T.z1);
            cnt[0] += bm ? (unsigned long long)NA : 0ull;
            cnt[1] += (unsigned long long)__popcll(bm) * (unsigned long long)NA;
        }
    }
}
template <int K, bool ZC>
__device__ __forceinline__ void spread_adds(double* ring, const TileAdds<SSh<K, ZC>::W>& T) {
    using S = SSh<K, ZC>;
    constexpr int W = S::W, NSL = S::NSL, NA = TileAdds<W>::NA;
    char* const rb = reinterpret_cast<char*>(ring);
    int sl = T.sl;
#pragma unroll
    for (int i2 = 0; i2 < W; ++i2) {
        char* const plane = rb + sl * (8 * S::PV);
        sl = sl + 1 == NSL ? 0 : sl + 1;
        // lanes whose plane is clipped or not owned sit it out (one exec mask per
        // plane: the edge anchors of a short z-piece reach mostly unowned planes)
        if (!(i2 >= T.z0 && i2 <= T.z1)) continue;
        const double w2 = T.wz[i2];
        // the values and addresses of a batch first, each in a register of its own
        // (the empty asm holds it there), then its adds back to back: otherwise
        // the compiler recycles one register pair, so that every ds_add_f64 waits
        // for its own multiply and the next multiply for the ds_add (IB_6, IB_4_W8:
        // batches of 8, 16, for the registers)
        constexpr int BT = W == 6 ? 8 : (W == 8 ? 16 : NA);
#pragma unroll
        for (int k0 = 0; k0 < NA; k0 += BT) {
            double v[BT];
            char* ad[BT];
#pragma unroll
            for (int k = 0; k < BT; ++k) {
                v[k] = T.P[k0 + k] * w2;
                ad[k] = plane + T.off[k0 + k];
                asm volatile("" ::"v"(v[k]));
            }
#pragma unroll
            for (int k = 0; k < BT; ++k) {
#if IBTK_LE_DIAG_SPREAD & 1  // diagnostic: no LDS adds (results wrong by design)
                asm volatile("" ::"v"(v[k]), "v"(ad[k]));
#else
                __hip_atomic_fetch_add(reinterpret_cast<double*>(ad[k]), v[k], __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_WORKGROUP);
#endif
            }
        }
    }
}
template <int K, bool CNT, bool ZC, typename Before>
__device__ __forceinline__ void spread_tiled(const Params& p, const CompDesc& cd, double* ring, const Cand& cdat,
                                             bool act, int a, int X0, int Y0, int zorg, int xlo, int xhi, int ylo,
                                             int yhi, int plo, int phi, double inv_h3, const double* inv_d, Clk& clk,
                                             unsigned long long* cnt, Before&& before) {
    TileAdds<SSh<K, ZC>::W> T;
    spread_setup<K, CNT, ZC>(p, cd, cdat, act, a, X0, Y0, zorg, xlo, xhi, ylo, yhi, plo, phi, inv_h3, inv_d, cnt,
                             before, T);
    clk.lap(2);
    spread_adds<K, ZC>(ring, T);
    clk.lap(3);
}

// Spread work item = (segment, column, component).  Owned points: the column's
// 32 x COLY (x, y) and planes [p0, p1) of the segment, intersected with the
// component's ghost box.  Anchor planes a in [p0-HI, p1-1-LO] reach them: the
// ring holds planes a+LO..a+HI (u_old, then accumulating) plus a+HI+1 in
// flight; plane a+LO is written back after anchor a and its slot takes plane
// a+HI+2.  The candidates of anchor a+1 are staged while anchor a is added.
// CNT: the counted launch of ibtk_le_ctx_count_adds (a kernel of its own name, so
// profiles of the product sweep do not average it in)
template <int K, bool LVL, bool CNT, bool ZC>
__global__ __launch_bounds__(SW) void k_spread_sweep(Params p) {
    using S = SSh<K, ZC>;
    constexpr int LO = S::LO, HI = S::HIE, NPL = S::NPL, FAM = S::FAM;  // HI: the ring's reach
    __shared__ double ring[S::NSL * S::PV];
    const int it = sweep_item(p, p.ncomp);
    if (it < 0) return;
    int c;
    SweepItem si;
    item_decode(p, it, c, si);
    c += p.comp0;  // the launch's components start at comp0 (launch_spread_sweep_t)
    const int col = si.col;
    const int lane = lane_id();
    ColGeom cg;
    CompDesc cd;
    const int* bs;
    item_patch<LVL>(p, si, c, cg, cd, bs);
    gdouble* const sorted_X = cur_sorted_X(p);
    const int ncx = cg.ncx;
    const int cx = col % ncx, cy = col / ncx;
    if (cx == 0 || cx == ncx - 1 || cy == 0 || cy == cg.ncy - 1) return;  // guard columns own no points
    const int X0 = cg.org[0] + cx * COLX, Y0 = cg.org[1] + cy * COLY;  // absolute
    const int zorg = cg.org[2];
    // owned, in-array ranges (column-local x/y, relative planes)
    const int xlo = max(cd.lo[0] - X0, 0), xhi = min(cd.hi[0] - X0, COLX - 1);
    const int ylo = max(cd.lo[1] - Y0, 0), yhi = min(cd.hi[1] - Y0, COLY - 1);
    const int plo = max(si.p0, cd.lo[2] - zorg), phi = min(si.p1 - 1, cd.hi[2] - zorg);
    if (xlo > xhi || ylo > yhi || plo > phi) return;
    if (p.zmode) {  // the planes the item owns (reads and writes)
        const bool inner = zorg + plo >= p.zlo && zorg + phi <= p.zhi;
        if (inner != (p.zmode == 1)) return;
    }
    // a closed-form kernel's component whose z frame is shifted by -dz/2 takes its
    // candidates by the anchor of that frame (anchors 0 .. nz, the boundaries cs_off_z;
    // see k_cand_write), which puts its stencil planes at a + [LO, HI - 1] as a key-frame one's
    const bool shz = FAM == 0 && !cd.zcell;
    static_assert(ZC || FAM != 0, "closed-form kernels: every component on the key-frame ring");
    const int nza = shz ? cg.nz + 1 : cg.nz;  // anchor planes of the component's stream
    const int afirst = max(plo - HI, 0), alast = min(phi - LO, nza - 1);
    // the item's stretch of its column's candidate stream (k_cand_stream, column-major
    // (patch, column, anchor) order): anchors afirst .. alast are [cs_off[ca0], cs_off[ca0 + nk])
    const int* const cs_offs = shz ? p.cs_off_z : p.cs_off;
    const int ca0 = (LVL ? (shz ? p.pd[si.patch].ca_base_z : p.pd[si.patch].bucket_base / NBAND) : 0) + col * nza + afirst;
    // no candidate reaches the item: u unchanged (zero_first: 0; zero_ghosts: ghosts 0)
    const bool any = cs_offs[ca0 + (alast - afirst + 1)] > cs_offs[ca0];
    // zero_ghosts (ibtk_le_zero_ghosts_spread): the owned points outside the component's
    // data box start from 0 instead of their values -- ibtk_le_zero_ghosts fused in
    const bool zg = p.zero_ghosts && !p.zero_first;
    int dlo[3], dhi[3];  // the unique points (patch box): ibtk_le_zero_ghosts zeroes the others
#pragma unroll
    for (int d = 0; d < 3; ++d) {
        dlo[d] = cd.ilower[d];
        dhi[d] = cd.iupper[d];
    }
    const bool xy_inner = X0 >= dlo[0] && X0 + COLX - 1 <= dhi[0] && Y0 >= dlo[1] && Y0 + COLY - 1 <= dhi[1];
    const bool z_inner = zorg + plo >= dlo[2] && zorg + phi <= dhi[2];
    if (!any && !p.zero_first && !(zg && !(xy_inner && z_inner))) return;
    const int nlast = p.nsorted - 1;
    // the lane's points of a plane: slot index lane + 64 k (tile-major, so the
    // staging stores and writeback loads are contiguous in LDS), their array
    // offsets (clamped into the array) and owned bits
    // (byte offsets in a plane through a buffer resource, plane_rsrc; a point the
    // item does not own has OFF_NONE: its load returns 0 and its store is dropped)
    unsigned loff[NPL];
    unsigned gmask = 0;  // zero_ghosts: bit k = the lane's point k is an x/y ghost point
#pragma unroll
    for (int k = 0; k < NPL; ++k) {
        int xl, yl;
        ring_xy(lane + k * SW, xl, yl);
        const bool own = xl >= xlo && xl <= xhi && yl >= ylo && yl <= yhi;
        loff[k] = own ? 8u * (unsigned)((X0 + xl - cd.lo[0]) + (Y0 + yl - cd.lo[1]) * (int)cd.s1) : OFF_NONE;
        const int gx = X0 + xl, gy = Y0 + yl;
        if (zg && (gx < dlo[0] || gx > dhi[0] || gy < dlo[1] || gy > dhi[1])) gmask |= 1u << k;
    }
    auto zghost = [&](int z) { return zorg + z < dlo[2] || zorg + z > dhi[2]; };
    const unsigned plane_bytes = (unsigned)(8 * cd.s2);
    auto plane_ptr = [&](int z) {  // relative plane z, clamped into the array
        const int zc = min(max(zorg + z, cd.lo[2]), cd.hi[2]);
        return plane_rsrc(cd.u + (int64_t)(zc - cd.lo[2]) * cd.s2, plane_bytes);
    };
    if (!any) {  // no candidate: zero_first, the owned points are 0; zero_ghosts, the owned ghosts
        for (int z = plo; z <= phi; ++z) {
            const auto pb = plane_ptr(z);
            const bool all = p.zero_first || zghost(z);
#pragma unroll
            for (int k = 0; k < NPL; ++k) buf_st(pb, (all || ((gmask >> k) & 1u)) ? loff[k] : OFF_NONE, 0.0);
        }
        return;
    }
    // candidate data of sorted position e
    auto cand_at = [&](int e, Cand& d) {
        e = min(max(e, 0), nlast);  // (an idle lane's stream entry may lie past the stream's end)
#if IBTK_LE_DIAG_SPREAD & 8  // diagnostic: no candidate loads
        d.X[0] = d.X[1] = d.X[2] = 0.5 + 1e-9 * e;
        d.V = 1.0;
        d.s = 0;
        return;
#endif
        const D3 xs = ld3(sorted_X + (int64_t)3 * e);
        d.X[0] = xs.v[0];
        d.X[1] = xs.v[1];
        d.X[2] = xs.v[2];
        d.V = p.sorted_F[(int64_t)c * p.nsorted + e];
        d.s = FAM == 2 ? p.sorted_s[e] : 0;
    };
    Clk clk;
    unsigned long long cnt[2] = {0ull, 0ull};  // CNT: wave-uniform totals of the item
    const double inv_h3 = 1.0 / p.h3;
    const double inv_d[3] = {1.0 / p.bg.dx[0], 1.0 / p.bg.dx[1], 1.0 / p.bg.dx[2]};
    // adds of the n <= 64 candidates held one per lane (lane j's anchor plane:
    // a - 1 for j < r, else a); `before` as for spread_tiled
    auto process = [&](int a, int r, int n, const Cand& mine, auto&& before) {
#if IBTK_LE_DIAG_SPREAD & 4  // diagnostic: no candidate work at all (the skeleton)
        asm volatile("" ::"v"(mine.X[0]), "v"(mine.X[1]), "v"(mine.X[2]), "v"(mine.V));
        before();
#else
        spread_tiled<K, CNT, ZC>(p, cd, ring, mine, lane < n, lane < r ? a - 1 : a, X0, Y0, zorg, xlo, xhi, ylo, yhi, plo, phi,
                             inv_h3, inv_d, clk, cnt, before);
#endif
    };
    auto nothing = [] {};
    // two full chunks of anchor a (a dense plane's middle chunks): both set up, then
    // the first's adds and the second's -- the adds in the order of two process calls
    constexpr bool PAIR = S::W <= 4;  // (wider stencils: the registers of two set-ups)
    auto process2 = [&](int a, const Cand& m0, const Cand& m1) {
#if IBTK_LE_DIAG_SPREAD & 4
        asm volatile("" ::"v"(m0.X[0]), "v"(m0.X[1]), "v"(m0.X[2]), "v"(m0.V));
        asm volatile("" ::"v"(m1.X[0]), "v"(m1.X[1]), "v"(m1.X[2]), "v"(m1.V));
        return;
#endif
        TileAdds<S::W> T0, T1;
        spread_setup<K, CNT, ZC>(p, cd, m0, true, a, X0, Y0, zorg, xlo, xhi, ylo, yhi, plo, phi, inv_h3, inv_d, cnt,
                                 nothing, T0);
        spread_setup<K, CNT, ZC>(p, cd, m1, true, a, X0, Y0, zorg, xlo, xhi, ylo, yhi, plo, phi, inv_h3, inv_d, cnt,
                                 nothing, T1);
        clk.lap(2);
        spread_adds<K, ZC>(ring, T0);
        spread_adds<K, ZC>(ring, T1);
        clk.lap(3);
    };
    // plane z -> registers (the lane's NPL points); registers -> ring slot.  A
    // plane the item does not own receives no adds and is not written back: its
    // slot's contents do not matter, so it is not read.
    auto plane_load = [&](int z, double* v) {
        if (z < plo || z > phi) return;
        if (p.zero_first || (zg && zghost(z))) {  // the owned points start from 0: nothing to read
#pragma unroll
            for (int k = 0; k < NPL; ++k) v[k] = 0.0;
            return;
        }
        const auto pb = plane_ptr(z);
#pragma unroll
        for (int k = 0; k < NPL; ++k) v[k] = buf_ld(pb, ((gmask >> k) & 1u) ? OFF_NONE : loff[k]);  // ghosts read 0
    };
    auto plane_put = [&](int z, const double* v) {
        double* sl = ring + sslot<S>(z) * S::PV;
#pragma unroll
        for (int k = 0; k < NPL; ++k) sl[lane + k * SW] = v[k];
    };
    // Writeback of plane z (owned points, ring -> array) in two halves: the slot is
    // read into registers before the slot is reused (a wave's LDS operations run in
    // order, so the put that follows needs no wait), the stores go out later.  A
    // plane the item does not own (or no plane, on: false) gets an empty resource
    // and its stores are dropped: every anchor step issues the same stores, so the
    // compiler's waits for later loads count them exactly instead of waiting for
    // the stores of a conditional path to complete.
    auto wb_read = [&](int z, double* v) {
        const double* sl = ring + sslot<S>(z) * S::PV;
#pragma unroll
        for (int k = 0; k < NPL; ++k) v[k] = sl[lane + k * SW];
    };
    auto wb_store = [&](int z, bool on, const double* v) {
        const int zc = min(max(zorg + z, cd.lo[2]), cd.hi[2]);
        const bool own = on && z >= plo && z <= phi;
        const auto pb = plane_rsrc(cd.u + (int64_t)(zc - cd.lo[2]) * cd.s2, own ? plane_bytes : 0u);
#pragma unroll
        for (int k = 0; k < NPL; ++k) buf_st(pb, loff[k], v[k]);  // not-owned points: dropped
    };

    // The candidates stream through 64-lane chunks across anchor planes.  Anchor
    // a's chunk 1 holds the r leftover candidates of anchor a-1 (its last r, in
    // lanes 0..r-1) and the first 64-r of a; full middle chunks of a follow;
    // a's last partial chunk is carried into a+1's chunk 1.  The ring holds the
    // planes of anchors a-1 and a: [a-1+LO, a+HI].
    // The candidates come from the column's candidate stream (k_cand_stream): the
    // sorted positions of the 11 candidate ranges of every anchor plane, anchor after
    // anchor, so that chunk 1 of an anchor is one contiguous piece of it, and the
    // anchor boundaries o(k) = cs_off[ca0 + k] (k = a - afirst).  Each step loads the
    // positions of chunk 1 two anchors ahead and the candidates of chunk 1 one anchor
    // ahead (from the positions loaded at the step before).
    clk.start(p.stamps != nullptr);
    const int* const cs_pos = p.cs_pos;
    const int cs_last = p.cs_total - 1;
    const int nk = alast - afirst + 1;  // anchors of the item; o(nk) ends its stream
    auto off_load = [&](int k) { return cs_offs[ca0 + min(k, nk)]; };
    auto pos_load = [&](int j) { return cs_pos[min(max(j, 0), cs_last)]; };
    // prologue: planes afirst+LO .. afirst+HI-1 into the ring; plane afirst+HI, the
    // anchor boundaries o(0) .. o(3), chunk 1 of afirst and the positions of chunk 1
    // of afirst + 1 into registers
    double pv[NPL] = {};
    for (int z = afirst + LO; z < afirst + HI; ++z) {
        plane_load(z, pv);
        plane_put(z, pv);
    }
    plane_load(afirst + HI, pv);
    int O0 = __builtin_amdgcn_readfirstlane(off_load(0)), O1 = __builtin_amdgcn_readfirstlane(off_load(1));
    int O2 = __builtin_amdgcn_readfirstlane(off_load(2)), O3 = __builtin_amdgcn_readfirstlane(off_load(3));
    int O4v = off_load(4);  // o(k + 4), in flight
    int R0 = 0;                                 // candidates of anchor k-1 carried into chunk 1 of k
    int N0 = min(O1 - O0, SW);                  // lanes of chunk 1 of k
    int R1 = (O1 - O0 - N0) % SW;               // carried into chunk 1 of k+1
    int N1 = R1 + min(SW - R1, O2 - O1);        // lanes of chunk 1 of k+1
    Cand nxt, nxt2;                             // chunk 1 of k, of k+1
    {
        const int e0 = pos_load(O0 + min(lane, max(N0 - 1, 0)));
        cand_at(e0, nxt);
    }
    int I1 = pos_load(O1 - R1 + min(lane, max(N1 - 1, 0)));  // positions of chunk 1 of k+1, in flight
    clk.lap(0);
    // One anchor step: plane a+HI from registers into the ring, plane a+HI+1 into
    // registers.  (Two anchors ahead through two register buffers measured the same,
    // 16.1 vs 16.3 ms on cfg4: the streams are not what waits.)
    auto anchor_step = [&](int a, const Cand& cur, Cand& nxt) __attribute__((always_inline)) {
        const int k = a - afirst;
        const int zw = a - 2 + LO;  // no anchor left reaches it: written back this step
        double wb[NPL];
        wb_read(zw, wb);       // its slot ...
        plane_put(a + HI, pv);  // ... takes plane a+HI
        // The step's inputs loaded at the previous step (chunk 1, the positions of the
        // next chunk 1, an anchor boundary) are waited for here, before this step issues
        // its own loads and stores.  Left to the compiler, the wait falls mid-step and is
        // vmcnt(0) (the loop-carried copy of a pending load): it then waits for this
        // step's prefetch and writeback too.  cfg4 spread sweep 15.0 -> 13.0 ms (round 5).
        asm volatile("" ::"v"(cur.X[0]), "v"(cur.X[1]), "v"(cur.X[2]), "v"(cur.V), "v"(I1), "v"(O4v));
        const int O4 = __builtin_amdgcn_readfirstlane(O4v);
        const int cur_r = R0, cur_n = N0;
        const int tCur = O1 - O0;
        const int h = min(SW - R0, tCur);   // a's candidates in chunk 1
        const int nmid = (tCur - h) / SW;   // full middle chunks
        const int r_a = R1;                 // carried into a+1: (tCur - h) % SW
        clk.lap(1);
        // prefetch: the candidates of chunk 1 of a+1 (positions I1), the positions of
        // chunk 1 of a+2 (a+1's last r, then a+2's first), the boundary o(k+5); plane a+HI+1
        int R2 = 0, N2 = 0;
        if (a + 1 <= alast) {
            cand_at(I1, nxt);
            const int t1 = O2 - O1;
            R2 = (t1 - min(SW - R1, t1)) % SW;
            N2 = R2 + min(SW - R2, O3 - O2);
            I1 = pos_load(O2 - R2 + min(lane, max(N2 - 1, 0)));
            O4v = off_load(k + 5);
            plane_load(a + HI + 1, pv);
        }
        const bool wbon = a >= afirst + 2;
        if (cur_n > 0) process(a, cur_r, cur_n, cur, [&] { wb_store(zw, wbon, wb); });
        else wb_store(zw, wbon, wb);
        if (nmid > 0) {  // dense planes: the full middle chunks, stream positions O0 + h + 64 m
            // chunk m + 1's candidates load while chunk m is added (a dense plane, e.g. a
            // sheet of markers, is hundreds of chunks of one wave); their positions a chunk earlier
            const int mbase = O0 + h + lane;
            Cand more, more2;
            cand_at(pos_load(mbase), more);
            int m = 0;
            if constexpr (PAIR) {
                // two chunks set up before either's adds (two independent chains of
                // set-up arithmetic per lane); their adds keep the chunk order.  The
                // positions of a pair are loaded while the pair before it is added.
                if (nmid > 1) cand_at(pos_load(mbase + SW), more2);
                int q2 = pos_load(mbase + SW * 2), q3 = pos_load(mbase + SW * 3);
                for (; m + 1 < nmid; m += 2) {
                    const Cand n0 = more, n1 = more2;
                    if (m + 2 < nmid) cand_at(q2, more);
                    if (m + 3 < nmid) cand_at(q3, more2);
                    q2 = pos_load(mbase + SW * (m + 4));
                    q3 = pos_load(mbase + SW * (m + 5));
                    process2(a, n0, n1);
                }
            }
            int q1 = pos_load(mbase + SW * (m + 1));
            for (; m < nmid; ++m) {
                const Cand now = more;
                if (m + 1 < nmid) cand_at(q1, more);
                q1 = pos_load(mbase + SW * (m + 2));
                process(a, 0, SW, now, nothing);
            }
        }
        if (a == alast && r_a > 0) {  // the last anchor's leftovers: stream O1 - r_a .. O1 - 1
            Cand last;
            cand_at(pos_load(O1 - r_a + min(lane, r_a - 1)), last);
            process(a, 0, r_a, last, nothing);
        }
        R0 = R1;
        N0 = N1;
        R1 = R2;
        N1 = N2;
        O0 = O1;
        O1 = O2;
        O2 = O3;
        O3 = O4;
        clk.lap(4);
    };
    for (int a = afirst; a <= alast; ++a) {
        anchor_step(a, nxt, nxt2);
        nxt = nxt2;
    }
    {
        double wb[NPL];
        wb_read(alast - 1 + LO, wb);
        wb_store(alast - 1 + LO, true, wb);
        wb_read(alast + LO, wb);
        wb_store(alast + LO, true, wb);
    }

    clk.lap(5);
    clk.flush(p, it);
    if constexpr (CNT) {
        if (lane == 0) {
            atomicAdd(p.nadd, cnt[0]);
            atomicAdd(p.nadd + 1, cnt[1]);
        }
    }
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
// Segment length: about IBTK_LE_SEG_ITEMS (column, segment) items over the
// patch, but no segment shorter than 32 planes (the z halo of a segment is HI-LO
// planes), and the patch's planes cut into segments of equal length (+-1).
// Equal lengths matter more than the length: a short last segment leaves the
// last XCD idle while the others carry its planes -- cfg4 at S = 128 (8 x 128 +
// 11 planes) and S = 141 (7 x 141 + 48) ran the sweeps 9-11 % slower than at
// S = 149 (profiles/r02seg); with equal segments 5-14 segments per patch are
// within a few per cent (profiles/r02seg2).
#ifndef IBTK_LE_SEG_ITEMS
#define IBTK_LE_SEG_ITEMS 16384
#endif
// Segments shorter than MIN_SEG planes are not cut: a segment re-reads HI - LO
// planes of z halo (interp) or anchors (spread), so a thin z-slab (8 GPUs: 139
// planes) keeps two segments of ~70 planes rather than five of 32 -- measured
// on rank 0's slab of an 8-way cfg4 split, 6.2 -> 5.5 ms per step
// (bench.py --solo-slab 8, profiles/r02v).
// A level's patches (64^3 on cfg5) take segments down to 32 planes: two per patch
// instead of one gives the clustered level twice the items to balance (cfg5
// 2.00e9 -> 2.14e9 marker-ops/s, spread sweep 3.41 -> 3.08 ms, profiles/r02z).
// A patch too narrow to give the chip work in long segments (fewer than
// SMALL_ITEMS (column, segment) pairs: cfg2's 128^3 sphere has 45 columns) takes
// segments down to 8 planes instead: its sweeps are latency-bound walks of one
// wave per item, not plane streams.
constexpr int MIN_SEG = 64, MIN_SEG_LEVEL = 32, SMALL_ITEMS = 1024, MIN_SEG_SMALL = 8;
void sweep_segments(const ColGeom& cg, int& S, int& nseg, int seg_items, bool level) {
    const int min_seg = level ? MIN_SEG_LEVEL : MIN_SEG;
    long long want = seg_items > 0 ? seg_items : IBTK_LE_SEG_ITEMS;
    long long s = ((long long)cg.nz * cg.ncol + want - 1) / want;
    if (s < min_seg && seg_items <= 0) {
        const long long ns = cg.nz / min_seg > 1 ? cg.nz / min_seg : 1;  // segments of >= min_seg planes
        s = (cg.nz + ns - 1) / ns;
    }
    const long long ncol_real = (long long)(cg.ncx > 2 ? cg.ncx - 2 : 1) * (cg.ncy > 2 ? cg.ncy - 2 : 1);
    if (!level && seg_items <= 0 && ncol_real * ((cg.nz + s - 1) / s) < SMALL_ITEMS) {
        const long long ns = (SMALL_ITEMS + ncol_real - 1) / ncol_real;
        s = (cg.nz + ns - 1) / ns;
        if (s < MIN_SEG_SMALL) s = MIN_SEG_SMALL;
    } else if (s < 32) {
        s = 32;
    }
    if (s > cg.nz) s = cg.nz;
    if (s < 1) s = 1;
    const long long ns = (cg.nz + s - 1) / s;  // segments of about s planes, equal (+-1)
    s = (cg.nz + ns - 1) / ns;
    S = (int)s;
    nseg = (cg.nz + S - 1) / S;
}

// Sweep item table.  A (column, segment) whose own markers exceed `target` is
// cut into sub-segments of its planes (at least NS planes each): a fibre bundle
// along z is then many items instead of one wave's serial walk.  Sub-items own
// disjoint planes, so every grid point still gets its contributions from one
// item.  The interp does not depend on the split (one lane sums a marker); the
// spread adds a point's contributions anchor by anchor in sorted order, but two
// candidates of one 64-lane chunk that hit the same point add in their step and
// lane order, and where the chunks start depends on the item's first anchor: so
// a different split can round a spread sum differently (fixed settings are
// bit-stable run to run; tests/test_gpu_items.py).  The interp
// item of a sub-segment sums the markers anchored in its planes; the spread
// item owns its planes and takes the candidates of the anchors reaching them
// (NS - 1 extra anchor planes per cut).
// (segment, column) pair j of the level -> its patch, column grid, segments
__device__ __forceinline__ void job_patch(const Params& p, int j, int& q, ColGeom& cg, int& S, int& nseg, int& j0,
                                          const int*& bs) {
    if (!p.pd) {
        q = 0;
        cg = p.cg;
        S = p.S;
        nseg = p.nseg;
        j0 = 0;
        bs = p.plane_start;
        return;
    }
    int lo = 0, hi = p.npatch - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (p.pd[mid].jbase <= j) lo = mid;
        else hi = mid - 1;
    }
    const PatchDesc& P = p.pd[lo];
    q = lo;
    cg = P.cg;
    S = P.S;
    nseg = P.nseg;
    j0 = P.jbase;
    bs = p.plane_start + P.bucket_base;
}

// The column of the i-th job of a segment: rows of columns in strips of `strip`
// (>= 1) column rows, x-major within a strip, so that the jobs that run together
// on an XCD include y-neighbours as well as x-neighbours (their shared halo rows
// and candidate ranges then come from L2); strip 1 is plain row-major order.
__device__ __forceinline__ int job_column(const ColGeom& cg, int i, int strip) {
    if (strip <= 1) return i;
    const int band = strip * cg.ncx;            // jobs per full strip
    const int sb = i / band, w = i - sb * band;
    const int rows = min(strip, cg.ncy - sb * strip);  // the last strip may be shorter
    const int cx = w / rows, cy = sb * strip + (w - cx * rows);
    return cy * cg.ncx + cx;
}

// load-based sub-segments of (column col, planes [a0, a1))
template <int K>
__device__ __forceinline__ int load_split(const ColGeom& cg, const int* bs, int col, int a0, int a1, int target,
                                          int min_piece, long& load) {
    constexpr int NS = KT<K>::HI - KT<K>::LO + 1;
    load = 0;
    for (int a = a0; a < a1; ++a) load += bs[bucket(cg, a, col, NBAND)] - bs[bucket(cg, a, col, 0)];
    const int maxsub = max((a1 - a0) / max(NS, min_piece > 0 ? min_piece : 8), 1);
    return (int)min((long)maxsub, max(1L, (load + target - 1) / target));
}
// The pieces of (column col, planes [a0, a1)) and whether they are heavy (own markers
// per piece above `heavy`: scheduled first).  A heavy (column, segment) -- clustered
// markers: a fibre bundle along the column, a sheet across it -- is cut finer, down to
// HEAVY_TARGET own markers and one plane per piece: its pieces are the sweeps' tail
// (cfg5: the spread's longest items were as long as the rest of the launch).  Uniform
// markers never qualify, so their items are unchanged.
constexpr int HEAVY_TARGET = 2048, HEAVY_MIN_PIECE = 1;
template <int K>
__device__ __forceinline__ int item_pieces(const Params& p, const ColGeom& cg, const int* bs, int col, int a0, int a1,
                                           int target, int heavy, long& load, bool& hv) {
    int n = load_split<K>(cg, bs, col, a0, a1, target, p.tune.min_piece, load);
    hv = load > (long)heavy * n;
    if (hv) {
        const int ht = p.tune.heavy_target > 0 ? p.tune.heavy_target : HEAVY_TARGET;
        const int hm = p.tune.heavy_min_piece > 0 ? p.tune.heavy_min_piece : HEAVY_MIN_PIECE;
        long l2;
        n = max(n, load_split<K>(cg, bs, col, a0, a1, ht, hm, l2));
        if (p.tune.heavy_first < 0) hv = false;  // cut finer, but in table order
    }
    return n;
}
// the plane cuts (ibtk_le_ctx_set_plane_window: sorted, relative) strictly inside (b0, b1)
__device__ __forceinline__ int cuts_inside(const Params& p, int b0, int b1) {
    int c = 0;
    for (int i = 0; i < p.ncut; ++i) c += p.cut[i] > b0 && p.cut[i] < b1;
    return c;
}

// nsub[j]: the light pieces of job j, nsub[njobs + j]: its heavy pieces (own
// markers per piece above `heavy`; they head the item table, see sweep_item)
template <int K>
__global__ __launch_bounds__(BLOCK) void k_item_counts(Params p, int target, int heavy, int* nsub) {
    if (p.items_skip && *p.items_skip == 0) return;  // nsub stands
    const int j = blockIdx.x * BLOCK + threadIdx.x;
    if (j >= p.njobs) return;
    int q, S, nseg, j0;
    ColGeom cg;
    const int* bs;
    job_patch(p, j, q, cg, S, nseg, j0, bs);
    const int jl = j - j0;
    const int seg = jl / cg.ncol, col = job_column(cg, jl - seg * cg.ncol, p.strip);
    const int a0 = seg * S, a1 = min(a0 + S, cg.nz), len = a1 - a0;
    long load;
    bool hv;
    const int n = item_pieces<K>(p, cg, bs, col, a0, a1, target, heavy, load, hv);
    int pieces = n;
    if (p.ncut)
        for (int k = 0; k < n; ++k) pieces += cuts_inside(p, a0 + (len * k) / n, a0 + (len * (k + 1)) / n);
    nsub[j] = hv ? 0 : pieces;
    nsub[p.njobs + j] = hv ? pieces : 0;
}
template <int K>
__global__ __launch_bounds__(BLOCK) void k_item_write(Params p, int target, int heavy, const int* nsub,
                                                      const int* start, SweepItem* tab, int* ntot) {
    if (p.items_skip && *p.items_skip == 0) return;  // the table stands
    const int j = blockIdx.x * BLOCK + threadIdx.x;
    if (j >= p.njobs) return;
    int q, S, nseg, j0;
    ColGeom cg;
    const int* bs;
    job_patch(p, j, q, cg, S, nseg, j0, bs);
    const int jl = j - j0;
    const int seg = jl / cg.ncol, col = job_column(cg, jl - seg * cg.ncol, p.strip);
    const int a0 = seg * S, a1 = min(a0 + S, cg.nz), len = a1 - a0;
    long load;
    bool hv;
    const int n = item_pieces<K>(p, cg, bs, col, a0, a1, target, heavy, load, hv);
    const int nj = p.njobs;
    const int nheavy = start[2 * nj - 1] + nsub[2 * nj - 1];
    int w = hv ? start[nj + j] : nheavy + start[j];
    for (int k = 0; k < n; ++k) {
        int b0 = a0 + (len * k) / n;
        const int b1 = a0 + (len * (k + 1)) / n;
        for (int i = 0; i < p.ncut; ++i)
            if (p.cut[i] > b0 && p.cut[i] < b1) {
                tab[w++] = SweepItem{col, b0, p.cut[i], q};
                b0 = p.cut[i];
            }
        tab[w++] = SweepItem{col, b0, b1, q};
    }
    if (j == nj - 1) {
        ntot[0] = nheavy + start[j] + nsub[j];
        ntot[1] = nheavy;
    }
}

static int grid8(long items) { return (int)((items + 7) & ~7L); }
// a sweep's grid: the items, the heavy items' rounding to 8 (sweep_item), and with
// block dealing over the XCDs (xcd_block > 0) a block of slack per XCD
static int sweep_grid(const Params& p, long items) {
    const int B = p.tune.xcd_block != 0 ? p.tune.xcd_block : XCD_BLOCK;
    const long per = p.item_bound > 0 ? items / p.item_bound : 1;
    return grid8(items + 8 + (B > 0 ? 8L * B * per : 0));
}

template <int K> hipError_t launch_item_table_t(const Params& p, int target, int heavy, int* nsub, int* start,
                                                SweepItem* tab, int* ntot, void* temp, size_t temp_bytes,
                                                hipStream_t s) {
    const int nj = p.njobs;
    if (nj <= 0) return hipMemsetAsync(ntot, 0, 2 * sizeof(int), s);
    hipLaunchKernelGGL(k_item_counts<K>, dim3((nj + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, s, p, target, heavy, nsub);
    hipError_t e = launch_scan(temp, temp_bytes, nsub, start, nj, s);  // light pieces
    if (e != hipSuccess) return e;
    e = launch_scan(temp, temp_bytes, nsub + nj, start + nj, nj, s);   // heavy pieces
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_item_write<K>, dim3((nj + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, s, p, target, heavy, nsub,
                       start, tab, ntot);
    return hipGetLastError();
}

template <int K> hipError_t launch_bin_col_t(const Params& p, int n, unsigned* keys, int* vals, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_bin_col<K>, dim3((n + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, s, p, n, keys, vals);
    return hipGetLastError();
}
__global__ __launch_bounds__(BLOCK) void k_bucket_init(int n, int nbuckets, int* first) {
    const int b = blockIdx.x * BLOCK + threadIdx.x;
    if (b <= nbuckets) first[b] = n;
}

template <int K>
hipError_t launch_gather_col_t(const Params& p, int n, int* ss, double* sx, const unsigned* skeys, int nbuckets,
                               int* first, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_bucket_init, dim3((nbuckets + 1 + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, s, n, nbuckets, first);
    hipLaunchKernelGGL(k_gather_col<K>, dim3((n + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, s, p, n, ss, sx, skeys,
                       nbuckets, first);
    return hipGetLastError();
}
template <int K>
hipError_t launch_interp_sweep_t(const Params& p, int n, hipStream_t s, hipEvent_t ev0, hipEvent_t ev1) {
    if (ev0) (void)hipEventRecord(ev0, s);
    const long items = (long)p.item_bound * p.ncomp;
    bool done = false;
    if constexpr (I3Sh<K>::fits) {
        // the three components of an item in one workgroup (k_interp3), on request
        if (items > 0 && !p.pd && p.ncomp == I3C && p.tune.interp3 > 0) {
            hipLaunchKernelGGL((k_interp3<K, I3WPC, I3PF>), dim3(sweep_grid(p, p.item_bound)), dim3(SW * I3C * I3WPC), 0,
                               s, p);
            done = true;
        }
    }
    if (items > 0 && !done) {
        const dim3 g(sweep_grid(p, items)), b(SW * IWAVES);
        if (p.pd && p.lvl_nbr) hipLaunchKernelGGL((k_interp_sweep<K, true, true>), g, b, 0, s, p);
        else if (p.pd) hipLaunchKernelGGL((k_interp_sweep<K, true>), g, b, 0, s, p);
        else hipLaunchKernelGGL((k_interp_sweep<K, false>), g, b, 0, s, p);
    }
    if (ev1) (void)hipEventRecord(ev1, s);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    if (n > 0) hipLaunchKernelGGL(k_interp_outside_col, dim3(64), dim3(BLOCK), 0, s, p, n);
    return hipGetLastError();
}
// sorted_F[c * n + e] = Q(qcomp_c, s(e)): the spread values in sorted order.
// REC3: three components that are a whole 24-byte Q record (Q_depth 3, qcomp
// 0, 1, 2: the side-centred force), read as one record per lane.
template <bool REC3>
__global__ __launch_bounds__(BLOCK) void k_gather_F_col(Params p, int n, double* out) {
    const int e = blockIdx.x * BLOCK + threadIdx.x;
    if (e >= n) return;
    const int s = p.sorted_s[e];
    // density-weighted spread: F ds rounded once, as LDataManager.cpp:446-451 forms it
    const double w = p.ds ? p.ds[s] : 1.0;
    if constexpr (REC3) {
        const D3 r = ld3(p.Qin + (int64_t)3 * s);
#pragma unroll
        for (int c = 0; c < 3; ++c) out[(int64_t)c * n + e] = p.ds ? r.v[c] * w : r.v[c];
    } else {
        for (int c = 0; c < p.ncomp; ++c) {
            const double v = p.Qin[(int64_t)p.Q_depth * s + p.comp[c].qcomp];
            out[(int64_t)c * n + e] = p.ds ? v * w : v;
        }
    }
}

hipError_t launch_gather_F(const Params& p, hipStream_t s) {
    if (p.nsorted > 0) {
        const bool rec3 = p.ncomp == 3 && p.Q_depth == 3 && p.comp[0].qcomp == 0 && p.comp[1].qcomp == 1 &&
                          p.comp[2].qcomp == 2;
        const dim3 g((p.nsorted + BLOCK - 1) / BLOCK), b(BLOCK);
        if (rec3) hipLaunchKernelGGL(k_gather_F_col<true>, g, b, 0, s, p, p.nsorted, const_cast<double*>(p.sorted_F));
        else hipLaunchKernelGGL(k_gather_F_col<false>, g, b, 0, s, p, p.nsorted, const_cast<double*>(p.sorted_F));
    }
    return hipGetLastError();
}
template <int K>
hipError_t launch_spread_sweep_t(const Params& p, hipStream_t s, hipEvent_t ev0, hipEvent_t ev1, bool gather) {
    if (gather)
        if (hipError_t e = launch_gather_F(p, s); e != hipSuccess) return e;
    if (ev0) (void)hipEventRecord(ev0, s);  // the events bracket the sweep kernels alone
    // One launch of every component.  Closed-form kernels run them all on the 5-slot
    // key-frame ring (ZC): a component whose z frame is shifted by -dz/2 reads its
    // candidates from the shifted-z stream (k_cand_z), anchored in its own frame, so its
    // planes sit at a + [LO, HI - 1] as a key-frame one's.  (r03j had the z-side component
    // on a 6-slot ring in a second launch: cfg4 spread 15.0 ms vs 14.2 all on 5 slots.)
    // Tabulated kernels keep the general ring.
    const long items = (long)p.item_bound * p.ncomp;
    if (items > 0) {
        Params q = p;
        q.comp0 = 0;
        const dim3 g(sweep_grid(q, items)), b(SW);
        constexpr bool ZC = KT<K>::FAM == 0;
        if (q.nadd) {
            if (q.pd) hipLaunchKernelGGL((k_spread_sweep<K, true, true, ZC>), g, b, 0, s, q);
            else hipLaunchKernelGGL((k_spread_sweep<K, false, true, ZC>), g, b, 0, s, q);
        } else {
            if (q.pd) hipLaunchKernelGGL((k_spread_sweep<K, true, false, ZC>), g, b, 0, s, q);
            else hipLaunchKernelGGL((k_spread_sweep<K, false, false, ZC>), g, b, 0, s, q);
        }
    }
    if (ev1) (void)hipEventRecord(ev1, s);
    return hipGetLastError();
}

#define IBTK_LE_DISPATCH_K(KV, CALL)                                 \
    switch (KV) {                                                    \
    case K_PIECEWISE_CONSTANT: return CALL<K_PIECEWISE_CONSTANT>;    \
    case K_DISCONTINUOUS_LINEAR: return CALL<K_DISCONTINUOUS_LINEAR>; \
    case K_PIECEWISE_LINEAR: return CALL<K_PIECEWISE_LINEAR>;        \
    case K_PIECEWISE_CUBIC: return CALL<K_PIECEWISE_CUBIC>;          \
    case K_IB_3: return CALL<K_IB_3>;                                \
    case K_IB_4: return CALL<K_IB_4>;                                \
    case K_IB_4_W8: return CALL<K_IB_4_W8>;                          \
    case K_IB_6: return CALL<K_IB_6>;                                \
    case K_BSPLINE_4: return CALL<K_BSPLINE_4>;                      \
    default: return nullptr;                                         \
    }

using ItemTabFn = hipError_t (*)(const Params&, int, int, int*, int*, SweepItem*, int*, void*, size_t, hipStream_t);
static ItemTabFn pick_item_table(int k) { IBTK_LE_DISPATCH_K(k, launch_item_table_t) }
hipError_t launch_item_table(int kernel, const Params& p, int target, int heavy, int* nsub, int* start, SweepItem* tab,
                             int* ntot, void* temp, size_t temp_bytes, hipStream_t s) {
    ItemTabFn f = pick_item_table(kernel);
    return f ? f(p, target, heavy, nsub, start, tab, ntot, temp, temp_bytes, s) : hipErrorInvalidValue;
}
using BinColFn = hipError_t (*)(const Params&, int, unsigned*, int*, hipStream_t);
using GatherColFn = hipError_t (*)(const Params&, int, int*, double*, const unsigned*, int, int*, hipStream_t);
using InterpSwFn = hipError_t (*)(const Params&, int, hipStream_t, hipEvent_t, hipEvent_t);
using SpreadSwFn = hipError_t (*)(const Params&, hipStream_t, hipEvent_t, hipEvent_t, bool);
static BinColFn pick_bin_col(int k) { IBTK_LE_DISPATCH_K(k, launch_bin_col_t) }
static GatherColFn pick_gather_col(int k) { IBTK_LE_DISPATCH_K(k, launch_gather_col_t) }
static InterpSwFn pick_interp_sweep(int k) { IBTK_LE_DISPATCH_K(k, launch_interp_sweep_t) }
static SpreadSwFn pick_spread_sweep(int k) { IBTK_LE_DISPATCH_K(k, launch_spread_sweep_t) }

hipError_t launch_bin_col(int kernel, const Params& p, int n, unsigned* keys, int* vals, hipStream_t s) {
    BinColFn f = pick_bin_col(kernel);
    return f ? f(p, n, keys, vals, s) : hipErrorInvalidValue;
}

// incremental re-binning (k_rekey .. k_rebin_scatter)
template <int K>
hipError_t launch_rekey_t(const Params& p, const RebinBufs& r, hipStream_t s) {
    if (r.n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_rekey<K>, dim3((r.n + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, s, p, r.n, r.kold, r.lsorted,
                       r.xcur, r.xa, r.xb, r.mbits, r.wcnt, r.cin, r.cout, KT<K>::FAM == 0 ? r.zbits : nullptr,
                       r.zst, r.epoch, r.nw, r.nbig);
    return hipGetLastError();
}
template <int K>
hipError_t launch_rebin_copy_t(const Params& p, const RebinBufs& r, hipStream_t s) {
    if (r.n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_rebin_copy<K>, dim3(RB_GRID), dim3(BLOCK), 0, s, p, r.n, r.wpre + r.nw, r.mbits, r.kold,
                       r.lsorted, r.xcur, r.xa, r.xb, r.knew, r.lold, KT<K>::FAM == 0 ? r.zst : nullptr);
    return hipGetLastError();
}
using RekeyFn = hipError_t (*)(const Params&, const RebinBufs&, hipStream_t);
static RekeyFn pick_rekey(int k) { IBTK_LE_DISPATCH_K(k, launch_rekey_t) }
static RekeyFn pick_rebin_copy(int k) { IBTK_LE_DISPATCH_K(k, launch_rebin_copy_t) }
hipError_t launch_rekey(int kernel, const Params& p, const RebinBufs& r, hipStream_t s) {
    RekeyFn f = pick_rekey(kernel);
    return f ? f(p, r, s) : hipErrorInvalidValue;
}
hipError_t launch_rebin_copy(int kernel, const Params& p, const RebinBufs& r, hipStream_t s) {
    RekeyFn f = pick_rebin_copy(kernel);
    return f ? f(p, r, s) : hipErrorInvalidValue;
}
static dim3 grid_of(long n) { return dim3((unsigned)((n + BLOCK - 1) / BLOCK)); }
int rebin_blocks(int nb) { return (int)(((long)nb + 2 + RB_BLK - 1) / RB_BLK); }
hipError_t launch_rebin_starts(const RebinBufs& r, hipStream_t s) {
    const int T_off = r.nw;
    const int* T = r.wpre + T_off;
    const int nblk = rebin_blocks(r.nb);
    int2* bsum = reinterpret_cast<int2*>(r.d);
    hipLaunchKernelGGL(k_rebin_bsum, dim3(nblk), dim3(BLOCK), 0, s, r.nb, r.cin, r.cout, T, bsum);
    hipLaunchKernelGGL(k_rebin_btop, dim3(1), dim3(BLOCK), 0, s, nblk, T, bsum);
    hipLaunchKernelGGL(k_rebin_bapply, dim3(nblk), dim3(BLOCK), 0, s, r.nb, r.cin, r.cout, r.os, T, bsum, r.ns,
                       r.mstart);
    return hipGetLastError();
}
hipError_t launch_rebin_movers(const RebinBufs& r, hipStream_t s) {
    const int* T = r.wpre + r.nw;
    if (r.n > 0)
        hipLaunchKernelGGL(k_rebin_append, grid_of(r.nw), dim3(BLOCK), 0, s, r.n, r.nw, r.mbits, r.knew, r.kold,
                           r.lold, r.mstart, r.cin, r.cout, r.mlist);
    hipLaunchKernelGGL(k_rebin_sort_small, dim3(RB_GRID), dim3(BLOCK), 0, s, r.nb, T, r.mstart, r.mlist, r.nbig,
                       r.big);
    hipLaunchKernelGGL(k_rebin_sort_big, dim3(1024), dim3(BLOCK), 0, s, r.nbig, r.big, r.mstart, r.mlist, r.scratch);
    hipLaunchKernelGGL(k_rebin_copy_big, dim3(1024), dim3(BLOCK), 0, s, r.nbig, r.big, r.mstart, r.scratch, r.mlist);
    return hipGetLastError();
}
hipError_t launch_rebin_scatter(const Params& p, const RebinBufs& r, hipStream_t s) {
    if (r.n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_rebin_scatter, dim3(RB_GRID), dim3(BLOCK), 0, s, p, r.n, r.nb, r.mbits, r.wpre, r.nw, r.knew,
                       r.lold, r.os, r.ns, r.mstart, r.mlist, r.sorted_l, r.sorted_key, r.sorted_s, r.xcur, r.xa, r.xb);
    hipLaunchKernelGGL(k_rebin_commit, dim3(RB_GRID), dim3(BLOCK), 0, s, r.nb, r.wpre + r.nw, r.ns,
                       const_cast<int*>(r.os), r.xcur, r.xa, r.xb, r.order_gen);
    return hipGetLastError();
}
hipError_t launch_gather_col(int kernel, const Params& p, int n, int* sorted_s, double* sorted_X,
                             const unsigned* sorted_key, int nbuckets, int* bucket_start, hipStream_t s) {
    GatherColFn f = pick_gather_col(kernel);
    return f ? f(p, n, sorted_s, sorted_X, sorted_key, nbuckets, bucket_start, s) : hipErrorInvalidValue;
}
hipError_t launch_interp_sweep(int kernel, const Params& p, int n, hipStream_t s, hipEvent_t ev0, hipEvent_t ev1) {
    InterpSwFn f = pick_interp_sweep(kernel);
    return f ? f(p, n, s, ev0, ev1) : hipErrorInvalidValue;
}
hipError_t launch_spread_sweep(int kernel, const Params& p, hipStream_t s, hipEvent_t ev0, hipEvent_t ev1,
                               bool gather) {
    SpreadSwFn f = pick_spread_sweep(kernel);
    return f ? f(p, s, ev0, ev1, gather) : hipErrorInvalidValue;
}

}  // namespace ibtk_le
