// le_interactor.cpp -- IBTK::LEInteractor facade (include/ibtk_le/LEInteractor.h)
// over the device-resident C-ABI.  Restates the C++ wrapper logic of
// ibtk/src/lagrangian/LEInteractor.cpp around the kernels:
//   * kernel-string checks (getStencilSize, :668-682) and ghost checks
//     (:2416-2426 interp; :2729-2745 spread, only at physical boundaries),
//   * depth checks of side/edge data (:767-771, :991-995, :1625-1629),
//   * buildLocalIndices (:3031-3108): the interior lists when box == patch box,
//     every list entry when box == the index set's ghost box,
//   * the X-only overloads (:1236-1546, 2094-2397; buildLocalIndices :3110-3139):
//     markers whose getCellIndex cell is in box, no periodic shifts,
//   * the std::vector overloads (:1148-1234, 2006-2092): the X-only form on the
//     vectors' data (staged through the device here),
//   * the per-axis frame shift of side/node/edge data (:1017-1053), which the
//     C-ABI applies for the SIDE/NODE/EDGE centerings.
// One lock is held from the list selection to the launch: the facade's scratch
// lists and bins are shared by every caller.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <mutex>
#include <string>

#include "../../include/ibtk_le.h"
#include "../../include/ibtk_le/LEInteractor.h"

namespace IBTK {
namespace {

struct DevScratch {
    void* p = nullptr;
    size_t cap = 0;
    void* get(size_t bytes) {
        if (bytes <= cap) return p;
        if (p) hipFree(p);
        p = nullptr;
        cap = 0;
        if (hipMalloc(&p, bytes) != hipSuccess)
            throw LEInteractorError(IBTK_LE_ERR_NOMEM, "LEInteractor: device allocation failed");
        cap = bytes;
        return p;
    }
};

struct Facade {
    std::mutex mu;
    int device = 0;
    void* stream = nullptr;
    ibtk_le_ctx ctx = nullptr;
    ibtk_le_markers m = nullptr;
    DevScratch filt, filt_xs, hostQ, hostX;  // box-filtered list (indices, shifts); staged std::vector data
    void ensure() {
        if (ctx) return;
        check(ibtk_le_ctx_create(device, stream, &ctx));
        check(ibtk_le_markers_create(ctx, &m));
    }
    static void check(int rc) {
        if (rc != IBTK_LE_OK) throw LEInteractorError(rc, ibtk_le_last_error());
    }
};

Facade& F() {
    static Facade f;
    return f;
}

int kernel_of(const std::string& name) {
    // the user-defined kernel function is read at every call, as the reference's
    // static pointer is (LEInteractor.cpp:651-652)
    if (name == "USER_DEFINED")
        Facade::check(ibtk_le_set_user_kernel(LEInteractor::s_kernel_fcn, LEInteractor::s_kernel_fcn_stencil_size));
    const int k = ibtk_le_kernel_from_name(name.c_str());
    if (k < 0)
        throw LEInteractorError(IBTK_LE_ERR_UNKNOWN_KERNEL,
                                "LEInteractor::getStencilSize()\n  Unknown kernel function " + name);
    return k;
}

ibtk_le_patch_geom make_geom(const PatchView& patch, const int* ghost) {
    ibtk_le_patch_geom g;
    std::memset(&g, 0, sizeof(g));
    g.ndim = patch.box.ndim;
    for (int d = 0; d < g.ndim; ++d) {
        g.ilower[d] = patch.box.lower[d];
        g.iupper[d] = patch.box.upper[d];
        g.gcw[d] = ghost[d];
        g.dx[d] = patch.dx[d];
        g.x_lower[d] = patch.x_lower[d];
        g.x_upper[d] = patch.x_upper[d];
    }
    return g;
}

bool touches_physical(const PatchView& p) {
    for (int d = 0; d < p.box.ndim; ++d)
        if (p.touches_physical_bdry[d][0] || p.touches_physical_bdry[d][1]) return true;
    return false;
}

int min_ghost(const int* g, int ndim) {
    int m = g[0];
    for (int d = 1; d < ndim; ++d) m = std::min(m, g[d]);
    return m;
}

// The Eulerian side of a call: centering, the arrays and their depth / ghosts.
struct Euler {
    int centering;
    double* arrays[3];
    int q_depth;
    const int* ghost;
};
Euler euler(const CellDataView& q) { return {IBTK_LE_CELL, {q.ptr, nullptr, nullptr}, q.depth, q.ghost}; }
Euler euler(const NodeDataView& q) { return {IBTK_LE_NODE, {q.ptr, nullptr, nullptr}, q.depth, q.ghost}; }
Euler euler(const SideDataView& q) { return {IBTK_LE_SIDE, {q.ptr[0], q.ptr[1], q.ptr[2]}, 1, q.ghost}; }
Euler euler(const EdgeDataView& q) { return {IBTK_LE_EDGE, {q.ptr[0], q.ptr[1], q.ptr[2]}, 1, q.ghost}; }

// the reference's depth checks (TBOX_ASSERT Q_depth == q depth for cell / node;
// TBOX_ERROR for side / edge data that is not NDIM-vector valued)
template <class V>
void check_depth(const V& q, int Q_depth, const char* who);
template <>
void check_depth(const CellDataView& q, int Q_depth, const char* who) {
    if (Q_depth != q.depth)
        throw LEInteractorError(IBTK_LE_ERR_DEPTH, std::string("LEInteractor::") + who + "(): Q depth != q depth");
}
template <>
void check_depth(const NodeDataView& q, int Q_depth, const char* who) {
    if (Q_depth != q.depth)
        throw LEInteractorError(IBTK_LE_ERR_DEPTH, std::string("LEInteractor::") + who + "(): Q depth != q depth");
}
template <>
void check_depth(const SideDataView& q, int Q_depth, const char* who) {
    if (Q_depth != q.box.ndim || q.depth != 1)
        throw LEInteractorError(IBTK_LE_ERR_DEPTH, std::string("LEInteractor::") + who + "():\n  side-centered " +
                                                       (who[0] == 'i' ? "interpolation" : "spreading") +
                                                       " requires vector-valued data.\n");
}
template <>
void check_depth(const EdgeDataView& q, int Q_depth, const char* who) {
    if (q.box.ndim != 3 || Q_depth != 3 || q.depth != 1)
        throw LEInteractorError(IBTK_LE_ERR_DEPTH, std::string("LEInteractor::") + who +
                                                       "():\n  edge-centered interpolation requires 3D "
                                                       "vector-valued data.\n");
}

// Where the call's markers come from: an index set and a box
// (buildLocalIndices, LEInteractor.cpp:3031-3108), or every marker of X whose
// cell lies in the box (:3110-3139).
struct Source {
    const LIndexSetBase* idx;  // null: the box filter of X
    int n_markers;             // box filter: markers in X
};

struct List {
    const int* idx;
    const double* xs;
    int n;
};

// f.mu held
List make_list(Facade& f, const Source& src, const PatchView& patch, const Box& box, const double* X) {
    if (src.idx) {
        const LIndexSetBase& idx = *src.idx;
        if (box == patch.box) return {idx.interior_local_indices, idx.interior_periodic_shifts, idx.n_interior};
        if (box == idx.ghost_box) return {idx.local_indices, idx.periodic_shifts, idx.n};
        // LEInteractor.cpp:3070-3106: the nodes of the set's cells inside the box, in
        // the set's order, each with its cell's periodic offset -- the entries of the
        // all-nodes list whose cell lies in the box
        if (!idx.cells)
            throw LEInteractorError(IBTK_LE_ERR_ARG,
                                    "LEInteractor: an index-set box other than the patch box or the ghost box needs "
                                    "the index set's cells (LIndexSetBase::cells)");
        if (idx.n <= 0) return {nullptr, nullptr, 0};
        const int nd = patch.box.ndim;
        int* oi = static_cast<int*>(f.filt.get(sizeof(int) * (size_t)idx.n));
        double* ox = static_cast<double*>(f.filt_xs.get(sizeof(double) * (size_t)nd * idx.n));
        int count = 0;
        Facade::check(ibtk_le_list_in_box(f.ctx, nd, idx.cells, idx.local_indices, idx.periodic_shifts, idx.n,
                                          box.lower, box.upper, oi, ox, idx.n, &count));
        return {oi, ox, count};
    }
    const int n = src.n_markers;
    if (n <= 0) return {nullptr, nullptr, 0};
    const int zero[3] = {0, 0, 0};
    const ibtk_le_patch_geom g = make_geom(patch, zero);
    int* out = static_cast<int*>(f.filt.get(sizeof(int) * (size_t)n));
    int count = 0;
    Facade::check(ibtk_le_box_index_list(f.ctx, &g, X, n, box.lower, box.upper, out, n, &count));
    return {out, nullptr, count};
}

// f.mu held
void interp_locked(Facade& f, const Euler& e, double* Q, int Q_depth, const double* X, int X_depth,
                   const Source& src, const PatchView& patch, const Box& box, const std::string& fcn) {
    const int k = kernel_of(fcn);
    f.ensure();
    const ibtk_le_patch_geom g = make_geom(patch, e.ghost);
    if (X_depth != g.ndim) throw LEInteractorError(IBTK_LE_ERR_DEPTH, "LEInteractor::interpolate(): X depth != NDIM");
    if (min_ghost(e.ghost, g.ndim) < ibtk_le_min_ghost_width(k))
        throw LEInteractorError(IBTK_LE_ERR_GHOST_WIDTH,
                                "LEInteractor::interpolate(): insufficient ghost cells:  kernel function = " + fcn);
    const List l = make_list(f, src, patch, box, X);
    if (l.n == 0) return;  // LEInteractor.cpp:885 (!local_indices.empty())
    if (k == IBTK_LE_KERNEL_USER_DEFINED) {  // LEInteractor.cpp:2688-2703
        Facade::check(ibtk_le_user_interp(f.ctx, e.centering, 0, &g, e.arrays, e.q_depth, Q, Q_depth, X, l.idx, l.xs, l.n));
        return;
    }
    Facade::check(ibtk_le_markers_bin(f.ctx, f.m, &g, k, X, l.idx, l.xs, l.n));
    Facade::check(ibtk_le_interp(f.ctx, f.m, k, e.centering, 0, &g, e.arrays, e.q_depth, Q, Q_depth, X));
}

void spread_locked(Facade& f, const Euler& e, const double* Q, int Q_depth, const double* X, int X_depth,
                   const Source& src, const PatchView& patch, const Box& box, const std::string& fcn) {
    const int k = kernel_of(fcn);
    f.ensure();
    const ibtk_le_patch_geom g = make_geom(patch, e.ghost);
    if (X_depth != g.ndim) throw LEInteractorError(IBTK_LE_ERR_DEPTH, "LEInteractor::spread(): X depth != NDIM");
    if (touches_physical(patch) && min_ghost(e.ghost, g.ndim) < ibtk_le_min_ghost_width(k))
        throw LEInteractorError(IBTK_LE_ERR_GHOST_WIDTH,
                                "LEInteractor::spread(): insufficient ghost cells at physical boundary:  kernel "
                                "function = " + fcn);
    const List l = make_list(f, src, patch, box, X);
    if (l.n == 0) return;
    if (k == IBTK_LE_KERNEL_USER_DEFINED) {  // LEInteractor.cpp:3007-3022
        Facade::check(ibtk_le_user_spread(f.ctx, e.centering, 0, &g, e.arrays, e.q_depth, Q, Q_depth, X, l.idx, l.xs, l.n));
        return;
    }
    Facade::check(ibtk_le_markers_bin(f.ctx, f.m, &g, k, X, l.idx, l.xs, l.n));
    Facade::check(ibtk_le_spread(f.ctx, f.m, k, e.centering, 0, &g, e.arrays, e.q_depth, Q, Q_depth, X));
}

template <class V>
void interp_any(const V& q, double* Q, int Q_depth, const double* X, int X_depth, const Source& src,
                const PatchView& patch, const Box& box, const std::string& fcn) {
    check_depth(q, Q_depth, "interpolate");
    Facade& f = F();
    std::lock_guard<std::mutex> lock(f.mu);
    interp_locked(f, euler(q), Q, Q_depth, X, X_depth, src, patch, box, fcn);
}

template <class V>
void spread_any(const V& q, const double* Q, int Q_depth, const double* X, int X_depth, const Source& src,
                const PatchView& patch, const Box& box, const std::string& fcn) {
    check_depth(q, Q_depth, "spread");
    Facade& f = F();
    std::lock_guard<std::mutex> lock(f.mu);
    spread_locked(f, euler(q), Q, Q_depth, X, X_depth, src, patch, box, fcn);
}

void check_sizes(int Q_size, int Q_depth, int X_size, int X_depth, const char* who) {
    if (Q_depth <= 0 || X_depth <= 0 || Q_size % Q_depth || X_size % X_depth || Q_size / Q_depth != X_size / X_depth)
        throw LEInteractorError(IBTK_LE_ERR_ARG, std::string("LEInteractor::") + who +
                                                     "(): Q_size / Q_depth != X_size / X_depth");
}

// std::vector forms: the host vectors staged through the device (interp copies
// Q in, so entries outside the box keep their values, and back out)
template <class V>
void interp_host(const V& q, std::vector<double>& Q, int Q_depth, const std::vector<double>& X, int X_depth,
                 const PatchView& patch, const Box& box, const std::string& fcn) {
    if (Q.empty()) return;  // LEInteractor.cpp:1157
    check_depth(q, Q_depth, "interpolate");
    check_sizes((int)Q.size(), Q_depth, (int)X.size(), X_depth, "interpolate");
    Facade& f = F();
    std::lock_guard<std::mutex> lock(f.mu);
    f.ensure();
    hipStream_t s = static_cast<hipStream_t>(f.stream);
    double* Qd = static_cast<double*>(f.hostQ.get(sizeof(double) * Q.size()));
    double* Xd = static_cast<double*>(f.hostX.get(sizeof(double) * X.size()));
    if (hipMemcpyAsync(Qd, Q.data(), sizeof(double) * Q.size(), hipMemcpyHostToDevice, s) != hipSuccess ||
        hipMemcpyAsync(Xd, X.data(), sizeof(double) * X.size(), hipMemcpyHostToDevice, s) != hipSuccess)
        throw LEInteractorError(IBTK_LE_ERR_DEVICE, "LEInteractor::interpolate(): host -> device copy failed");
    interp_locked(f, euler(q), Qd, Q_depth, Xd, X_depth, Source{nullptr, (int)(X.size() / X_depth)}, patch, box,
                  fcn);
    if (hipMemcpyAsync(Q.data(), Qd, sizeof(double) * Q.size(), hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
        throw LEInteractorError(IBTK_LE_ERR_DEVICE, "LEInteractor::interpolate(): device -> host copy failed");
}

template <class V>
void spread_host(const V& q, const std::vector<double>& Q, int Q_depth, const std::vector<double>& X, int X_depth,
                 const PatchView& patch, const Box& box, const std::string& fcn) {
    if (Q.empty()) return;  // LEInteractor.cpp:2015
    check_depth(q, Q_depth, "spread");
    check_sizes((int)Q.size(), Q_depth, (int)X.size(), X_depth, "spread");
    Facade& f = F();
    std::lock_guard<std::mutex> lock(f.mu);
    f.ensure();
    hipStream_t s = static_cast<hipStream_t>(f.stream);
    double* Qd = static_cast<double*>(f.hostQ.get(sizeof(double) * Q.size()));
    double* Xd = static_cast<double*>(f.hostX.get(sizeof(double) * X.size()));
    if (hipMemcpyAsync(Qd, Q.data(), sizeof(double) * Q.size(), hipMemcpyHostToDevice, s) != hipSuccess ||
        hipMemcpyAsync(Xd, X.data(), sizeof(double) * X.size(), hipMemcpyHostToDevice, s) != hipSuccess)
        throw LEInteractorError(IBTK_LE_ERR_DEVICE, "LEInteractor::spread(): host -> device copy failed");
    spread_locked(f, euler(q), Qd, Q_depth, Xd, X_depth, Source{nullptr, (int)(X.size() / X_depth)}, patch, box,
                  fcn);
    // the staged arrays are reused by the next call: wait for this one
    if (hipStreamSynchronize(s) != hipSuccess)
        throw LEInteractorError(IBTK_LE_ERR_DEVICE, "LEInteractor::spread(): stream failure");
}

}  // namespace

double (*LEInteractor::s_kernel_fcn)(double r) = &ibtk_le_ib4_kernel_fcn;  // LEInteractor.cpp:651
int LEInteractor::s_kernel_fcn_stencil_size = 4;

void LEInteractor::setFromDatabase(const void*) {}
void LEInteractor::printClassData(std::ostream& os) { os << "LEInteractor::printClassData():\n"; }
int LEInteractor::getStencilSize(const std::string& kernel_fcn) { return ibtk_le_stencil_size(kernel_of(kernel_fcn)); }
int LEInteractor::getMinimumGhostWidth(const std::string& kernel_fcn) {
    return ibtk_le_min_ghost_width(kernel_of(kernel_fcn));
}

void LEInteractor::setStream(int device, void* hip_stream) {
    Facade& f = F();
    std::lock_guard<std::mutex> lock(f.mu);
    f.device = device;
    f.stream = hip_stream;
    if (f.ctx) Facade::check(ibtk_le_ctx_set_stream(f.ctx, hip_stream));
}

void LEInteractor::synchronize() {
    Facade& f = F();
    std::lock_guard<std::mutex> lock(f.mu);
    if (f.ctx) Facade::check(ibtk_le_ctx_synchronize(f.ctx));
}

// The four argument forms, each for Cell / Node / Side / Edge data.
#define IBTK_LE_FACADE_OVERLOADS(VIEW)                                                                               \
    void LEInteractor::interpolate(LDataView Q, LDataView X, const LIndexSetBase& idx, const VIEW& q,                \
                                   const PatchView& patch, const Box& box, const int*, const std::string& fcn) {     \
        interp_any(q, Q.ptr, Q.depth, X.ptr, X.depth, Source{&idx, 0}, patch, box, fcn);                             \
    }                                                                                                                \
    void LEInteractor::interpolate(double* Q, int Q_depth, const double* X, int X_depth, const LIndexSetBase& idx,   \
                                   const VIEW& q, const PatchView& patch, const Box& box, const int*,                \
                                   const std::string& fcn) {                                                         \
        interp_any(q, Q, Q_depth, X, X_depth, Source{&idx, 0}, patch, box, fcn);                                     \
    }                                                                                                                \
    void LEInteractor::interpolate(std::vector<double>& Q, int Q_depth, const std::vector<double>& X, int X_depth,   \
                                   const VIEW& q, const PatchView& patch, const Box& box, const std::string& fcn) {  \
        interp_host(q, Q, Q_depth, X, X_depth, patch, box, fcn);                                                     \
    }                                                                                                                \
    void LEInteractor::interpolate(double* Q, int Q_size, int Q_depth, const double* X, int X_size, int X_depth,     \
                                   const VIEW& q, const PatchView& patch, const Box& box, const std::string& fcn) {  \
        check_sizes(Q_size, Q_depth, X_size, X_depth, "interpolate");                                                \
        interp_any(q, Q, Q_depth, X, X_depth, Source{nullptr, X_size / X_depth}, patch, box, fcn);                   \
    }                                                                                                                \
    void LEInteractor::spread(const VIEW& q, LDataView Q, LDataView X, const LIndexSetBase& idx,                     \
                              const PatchView& patch, const Box& box, const int*, const std::string& fcn) {          \
        spread_any(q, Q.ptr, Q.depth, X.ptr, X.depth, Source{&idx, 0}, patch, box, fcn);                             \
    }                                                                                                                \
    void LEInteractor::spread(const VIEW& q, const double* Q, int Q_depth, const double* X, int X_depth,             \
                              const LIndexSetBase& idx, const PatchView& patch, const Box& box, const int*,          \
                              const std::string& fcn) {                                                              \
        spread_any(q, Q, Q_depth, X, X_depth, Source{&idx, 0}, patch, box, fcn);                                     \
    }                                                                                                                \
    void LEInteractor::spread(const VIEW& q, const std::vector<double>& Q, int Q_depth,                              \
                              const std::vector<double>& X, int X_depth, const PatchView& patch, const Box& box,     \
                              const std::string& fcn) {                                                              \
        spread_host(q, Q, Q_depth, X, X_depth, patch, box, fcn);                                                     \
    }                                                                                                                \
    void LEInteractor::spread(const VIEW& q, const double* Q, int Q_size, int Q_depth, const double* X, int X_size,  \
                              int X_depth, const PatchView& patch, const Box& box, const std::string& fcn) {         \
        check_sizes(Q_size, Q_depth, X_size, X_depth, "spread");                                                     \
        spread_any(q, Q, Q_depth, X, X_depth, Source{nullptr, X_size / X_depth}, patch, box, fcn);                   \
    }

IBTK_LE_FACADE_OVERLOADS(CellDataView)
IBTK_LE_FACADE_OVERLOADS(NodeDataView)
IBTK_LE_FACADE_OVERLOADS(SideDataView)
IBTK_LE_FACADE_OVERLOADS(EdgeDataView)
#undef IBTK_LE_FACADE_OVERLOADS

}  // namespace IBTK
