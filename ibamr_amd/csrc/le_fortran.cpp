// le_fortran.cpp -- drop-in replacements for the Fortran kernels IBAMR links
// against: lagrangian_<kernel>_{interp,spread}{2,3}d_, with the exact by-reference
// argument lists LEInteractor.cpp:68-619 declares (IBTK_FC_FUNC_: lowercase,
// trailing underscore).  Host memory in, host memory out: each call copies the
// patch array and the listed markers to the GPU, runs the HIP kernels through the
// device-resident C-ABI and copies the results back.
//
// Semantics vs the Fortran:
//  * interp writes V(:, s) for every listed s; if s is listed more than once the
//    last entry wins, as in the Fortran's sequential l-loop.
//  * spread sums each grid point's contributions in the canonical (binned) order
//    of the list rather than the given order; results agree with the Fortran to
//    rounding (<= 1e-12 normwise) and are bit-stable run to run.  Callers that
//    already pass a cell-sorted list (LDataManager's numbering) get the same
//    per-point order as the Fortran.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>

#include "../../include/ibtk_le.h"
#include "../../include/ibtk_le_fortran.h"
#include "le_internal.h"

namespace {

struct Dev {
    void* p = nullptr;
    size_t cap = 0;
    bool ensure(size_t b) {
        if (b <= cap) return true;
        if (p) hipFree(p);
        p = nullptr;
        cap = 0;
        if (hipMalloc(&p, b + b / 8 + 64) != hipSuccess) return false;
        cap = b + b / 8 + 64;
        return true;
    }
};

struct ShimState {
    std::mutex mu;
    ibtk_le_ctx ctx = nullptr;
    ibtk_le_markers markers = nullptr;
    Dev u, X, idx, xs, V;
    bool init() {
        if (ctx) return true;
        if (ibtk_le_ctx_create(0, nullptr, &ctx) != IBTK_LE_OK) return false;
        if (ibtk_le_markers_create(ctx, &markers) != IBTK_LE_OK) return false;
        return true;
    }
};

ShimState& state() {
    static ShimState s;
    return s;
}

[[noreturn]] void die(const char* where) {
    // The reference aborts through TBOX_ERROR; the Fortran ABI has no status
    // return, so the shim does the same.
    std::fprintf(stderr, "ibtk_le %s: %s\n", where, ibtk_le_last_error());
    std::abort();
}

#define CHK(expr, where)                          \
    do {                                          \
        if ((expr) != IBTK_LE_OK) die(where);     \
    } while (0)
#define HCHK(expr, where)                                                                   \
    do {                                                                                    \
        hipError_t _e = (expr);                                                             \
        if (_e != hipSuccess) {                                                             \
            std::fprintf(stderr, "ibtk_le %s: %s\n", where, hipGetErrorString(_e));         \
            std::abort();                                                                   \
        }                                                                                   \
    } while (0)

// One depth-`depth` patch-array call.  `ilo/ihi` is the data box the Fortran
// received (cell box, or side/node box of one axis), `nugc` its ghost width,
// `x_lower` the (already frame-shifted) lower corner: exactly a cell-centred
// array of that box, so the shim runs the CELL centering with depth components.
void host_call(bool spread, int kernel, int ndim, const double* dx, const double* x_lower, const double* x_upper,
               int depth, int axis, const int* ilo, const int* ihi, const int* nugc, double* u, const int* indices,
               const double* Xshift, int nindices, const double* X, double* V) {
    if (nindices <= 0) return;
    ShimState& S = state();
    std::lock_guard<std::mutex> lock(S.mu);
    if (!S.init()) die("context");
    ibtk_le_patch_geom g;
    std::memset(&g, 0, sizeof(g));
    g.ndim = ndim;
    size_t npts = 1;
    for (int d = 0; d < ndim; ++d) {
        g.ilower[d] = ilo[d];
        g.iupper[d] = ihi[d];
        g.gcw[d] = nugc[d];
        g.dx[d] = dx[d];
        g.x_lower[d] = x_lower[d];
        g.x_upper[d] = x_upper[d];
        npts *= (size_t)(ihi[d] - ilo[d] + 1 + 2 * nugc[d]);
    }
    // list (interp: keep the last occurrence of each marker)
    std::vector<int> lidx(indices, indices + nindices);
    std::vector<double> lxs(Xshift, Xshift + (size_t)ndim * nindices);
    int nmark = 0;
    for (int l = 0; l < nindices; ++l) nmark = std::max(nmark, lidx[l] + 1);
    if (!spread) {
        std::vector<char> seen(nmark, 0);
        std::vector<int> keep;
        keep.reserve(nindices);
        for (int l = nindices - 1; l >= 0; --l)
            if (!seen[lidx[l]]) {
                seen[lidx[l]] = 1;
                keep.push_back(l);
            }
        std::reverse(keep.begin(), keep.end());
        if ((int)keep.size() != nindices) {
            std::vector<int> i2;
            std::vector<double> x2;
            for (int l : keep) {
                i2.push_back(lidx[l]);
                for (int d = 0; d < ndim; ++d) x2.push_back(lxs[(size_t)ndim * l + d]);
            }
            lidx.swap(i2);
            lxs.swap(x2);
        }
    }
    const int n = (int)lidx.size();
    const size_t ub = sizeof(double) * npts * depth;
    const size_t Xb = sizeof(double) * (size_t)ndim * nmark;
    const size_t Vb = sizeof(double) * (size_t)depth * nmark;
    if (!S.u.ensure(ub) || !S.X.ensure(Xb) || !S.idx.ensure(sizeof(int) * n) ||
        !S.xs.ensure(sizeof(double) * (size_t)ndim * n) || !S.V.ensure(Vb))
        die("device allocation");
    HCHK(hipMemcpy(S.u.p, u, ub, hipMemcpyHostToDevice), "H2D u");
    HCHK(hipMemcpy(S.X.p, X, Xb, hipMemcpyHostToDevice), "H2D X");
    HCHK(hipMemcpy(S.idx.p, lidx.data(), sizeof(int) * n, hipMemcpyHostToDevice), "H2D indices");
    HCHK(hipMemcpy(S.xs.p, lxs.data(), sizeof(double) * (size_t)ndim * n, hipMemcpyHostToDevice), "H2D Xshift");
    HCHK(hipMemcpy(S.V.p, V, Vb, hipMemcpyHostToDevice), "H2D V");
    CHK(ibtk_le_markers_bin(S.ctx, S.markers, &g, kernel, (const double*)S.X.p, (const int*)S.idx.p,
                            (const double*)S.xs.p, n),
        "bin");
    double* q[1] = {(double*)S.u.p};
    if (spread) {
        CHK(ibtk_le_spread(S.ctx, S.markers, kernel, IBTK_LE_CELL, axis, &g, q, depth, (const double*)S.V.p, depth,
                           (const double*)S.X.p),
            "spread");
    } else {
        // the Fortran itself does not check ghost widths (the C++ wrapper does,
        // LEInteractor.cpp:2416): call the kernels without that check
        CHK(ibtk_le::interp_impl(S.ctx, S.markers, kernel, IBTK_LE_CELL, axis, &g, q, depth, (double*)S.V.p, depth,
                                 (const double*)S.X.p, /*check_ghosts=*/false),
            "interp");
    }
    CHK(ibtk_le_ctx_synchronize(S.ctx), "kernel");
    if (spread) HCHK(hipMemcpy(u, S.u.p, ub, hipMemcpyDeviceToHost), "D2H u");
    else HCHK(hipMemcpy(V, S.V.p, Vb, hipMemcpyDeviceToHost), "D2H V");
}

}  // namespace

// ---------------------------------------------------------------------------
// symbol generators
// ---------------------------------------------------------------------------
#define IBTK_LE_INTERP3D(NAME, KID)                                                                                   \
    extern "C" void NAME(const double* dx, const double* x_lower, const double* x_upper, const int* depth,         \
                         const int* ilower0, const int* iupper0, const int* ilower1, const int* iupper1,            \
                         const int* ilower2, const int* iupper2, const int* nugc0, const int* nugc1,                \
                         const int* nugc2, const double* u, const int* indices, const double* Xshift,               \
                         const int* nindices, const double* X, double* V) {                                          \
        const int lo[3] = {*ilower0, *ilower1, *ilower2}, hi[3] = {*iupper0, *iupper1, *iupper2};                   \
        const int g[3] = {*nugc0, *nugc1, *nugc2};                                                                  \
        host_call(false, KID, 3, dx, x_lower, x_upper, *depth, 0, lo, hi, g, const_cast<double*>(u), indices,     \
                  Xshift, *nindices, X, V);                                                                         \
    }
#define IBTK_LE_SPREAD3D(NAME, KID)                                                                                   \
    extern "C" void NAME(const double* dx, const double* x_lower, const double* x_upper, const int* depth,         \
                         const int* indices, const double* Xshift, const int* nindices, const double* X,            \
                         const double* V, const int* ilower0, const int* iupper0, const int* ilower1,               \
                         const int* iupper1, const int* ilower2, const int* iupper2, const int* nugc0,              \
                         const int* nugc1, const int* nugc2, double* u) {                                           \
        const int lo[3] = {*ilower0, *ilower1, *ilower2}, hi[3] = {*iupper0, *iupper1, *iupper2};                   \
        const int g[3] = {*nugc0, *nugc1, *nugc2};                                                                  \
        host_call(true, KID, 3, dx, x_lower, x_upper, *depth, 0, lo, hi, g, u, indices, Xshift, *nindices, X,     \
                  const_cast<double*>(V));                                                                          \
    }
#define IBTK_LE_INTERP2D(NAME, KID)                                                                                   \
    extern "C" void NAME(const double* dx, const double* x_lower, const double* x_upper, const int* depth,         \
                         const int* ilower0, const int* iupper0, const int* ilower1, const int* iupper1,            \
                         const int* nugc0, const int* nugc1, const double* u, const int* indices,                   \
                         const double* Xshift, const int* nindices, const double* X, double* V) {                    \
        const int lo[2] = {*ilower0, *ilower1}, hi[2] = {*iupper0, *iupper1}, g[2] = {*nugc0, *nugc1};              \
        host_call(false, KID, 2, dx, x_lower, x_upper, *depth, 0, lo, hi, g, const_cast<double*>(u), indices,     \
                  Xshift, *nindices, X, V);                                                                         \
    }
#define IBTK_LE_SPREAD2D(NAME, KID)                                                                                   \
    extern "C" void NAME(const double* dx, const double* x_lower, const double* x_upper, const int* depth,         \
                         const int* indices, const double* Xshift, const int* nindices, const double* X,            \
                         const double* V, const int* ilower0, const int* iupper0, const int* ilower1,               \
                         const int* iupper1, const int* nugc0, const int* nugc1, double* u) {                       \
        const int lo[2] = {*ilower0, *ilower1}, hi[2] = {*iupper0, *iupper1}, g[2] = {*nugc0, *nugc1};              \
        host_call(true, KID, 2, dx, x_lower, x_upper, *depth, 0, lo, hi, g, u, indices, Xshift, *nindices, X,     \
                  const_cast<double*>(V));                                                                          \
    }
// DISCONTINUOUS_LINEAR carries `axis` after `depth` (LEInteractor.cpp:200-262)
#define IBTK_LE_DL_INTERP3D(NAME, KID)                                                                                \
    extern "C" void NAME(const double* dx, const double* x_lower, const double* x_upper, const int* depth,         \
                         const int* axis, const int* ilower0, const int* iupper0, const int* ilower1,               \
                         const int* iupper1, const int* ilower2, const int* iupper2, const int* nugc0,              \
                         const int* nugc1, const int* nugc2, const double* u, const int* indices,                   \
                         const double* Xshift, const int* nindices, const double* X, double* V) {                    \
        const int lo[3] = {*ilower0, *ilower1, *ilower2}, hi[3] = {*iupper0, *iupper1, *iupper2};                   \
        const int g[3] = {*nugc0, *nugc1, *nugc2};                                                                  \
        host_call(false, KID, 3, dx, x_lower, x_upper, *depth, *axis, lo, hi, g, const_cast<double*>(u), indices, \
                  Xshift, *nindices, X, V);                                                                         \
    }
#define IBTK_LE_DL_SPREAD3D(NAME, KID)                                                                                \
    extern "C" void NAME(const double* dx, const double* x_lower, const double* x_upper, const int* depth,         \
                         const int* axis, const int* indices, const double* Xshift, const int* nindices,            \
                         const double* X, const double* V, const int* ilower0, const int* iupper0,                  \
                         const int* ilower1, const int* iupper1, const int* ilower2, const int* iupper2,            \
                         const int* nugc0, const int* nugc1, const int* nugc2, double* u) {                         \
        const int lo[3] = {*ilower0, *ilower1, *ilower2}, hi[3] = {*iupper0, *iupper1, *iupper2};                   \
        const int g[3] = {*nugc0, *nugc1, *nugc2};                                                                  \
        host_call(true, KID, 3, dx, x_lower, x_upper, *depth, *axis, lo, hi, g, u, indices, Xshift, *nindices, X, \
                  const_cast<double*>(V));                                                                          \
    }
#define IBTK_LE_DL_INTERP2D(NAME, KID)                                                                                \
    extern "C" void NAME(const double* dx, const double* x_lower, const double* x_upper, const int* depth,         \
                         const int* axis, const int* ilower0, const int* iupper0, const int* ilower1,               \
                         const int* iupper1, const int* nugc0, const int* nugc1, const double* u,                   \
                         const int* indices, const double* Xshift, const int* nindices, const double* X,            \
                         double* V) {                                                                               \
        const int lo[2] = {*ilower0, *ilower1}, hi[2] = {*iupper0, *iupper1}, g[2] = {*nugc0, *nugc1};              \
        host_call(false, KID, 2, dx, x_lower, x_upper, *depth, *axis, lo, hi, g, const_cast<double*>(u), indices, \
                  Xshift, *nindices, X, V);                                                                         \
    }
#define IBTK_LE_DL_SPREAD2D(NAME, KID)                                                                                \
    extern "C" void NAME(const double* dx, const double* x_lower, const double* x_upper, const int* depth,         \
                         const int* axis, const int* indices, const double* Xshift, const int* nindices,            \
                         const double* X, const double* V, const int* ilower0, const int* iupper0,                  \
                         const int* ilower1, const int* iupper1, const int* nugc0, const int* nugc1, double* u) {   \
        const int lo[2] = {*ilower0, *ilower1}, hi[2] = {*iupper0, *iupper1}, g[2] = {*nugc0, *nugc1};              \
        host_call(true, KID, 2, dx, x_lower, x_upper, *depth, *axis, lo, hi, g, u, indices, Xshift, *nindices, X, \
                  const_cast<double*>(V));                                                                          \
    }

#define IBTK_LE_ALL(kname, KID)                          \
    IBTK_LE_INTERP3D(lagrangian_##kname##_interp3d_, KID) \
    IBTK_LE_SPREAD3D(lagrangian_##kname##_spread3d_, KID) \
    IBTK_LE_INTERP2D(lagrangian_##kname##_interp2d_, KID) \
    IBTK_LE_SPREAD2D(lagrangian_##kname##_spread2d_, KID)

IBTK_LE_ALL(piecewise_constant, ibtk_le::K_PIECEWISE_CONSTANT)
IBTK_LE_ALL(piecewise_linear, ibtk_le::K_PIECEWISE_LINEAR)
IBTK_LE_ALL(piecewise_cubic, ibtk_le::K_PIECEWISE_CUBIC)
IBTK_LE_ALL(ib_3, ibtk_le::K_IB_3)
IBTK_LE_ALL(ib_4, ibtk_le::K_IB_4)
IBTK_LE_ALL(ib_4_w8, ibtk_le::K_IB_4_W8)
IBTK_LE_ALL(ib_6, ibtk_le::K_IB_6)
IBTK_LE_DL_INTERP3D(lagrangian_discontinuous_linear_interp3d_, ibtk_le::K_DISCONTINUOUS_LINEAR)
IBTK_LE_DL_SPREAD3D(lagrangian_discontinuous_linear_spread3d_, ibtk_le::K_DISCONTINUOUS_LINEAR)
IBTK_LE_DL_INTERP2D(lagrangian_discontinuous_linear_interp2d_, ibtk_le::K_DISCONTINUOUS_LINEAR)
IBTK_LE_DL_SPREAD2D(lagrangian_discontinuous_linear_spread2d_, ibtk_le::K_DISCONTINUOUS_LINEAR)
