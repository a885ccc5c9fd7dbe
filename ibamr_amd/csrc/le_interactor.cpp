// le_interactor.cpp -- IBTK::LEInteractor facade (include/ibtk_le/LEInteractor.h)
// over the device-resident C-ABI.  Restates the C++ wrapper logic of
// ibtk/src/lagrangian/LEInteractor.cpp around the kernels:
//   * kernel-string checks (getStencilSize, :668-682) and ghost checks
//     (:2416-2426 interp; :2729-2745 spread, only at physical boundaries),
//   * depth checks of side/edge data (:767-771, :991-995, :1625-1629),
//   * buildLocalIndices (:3031-3108): the interior lists when box == patch box,
//     every list entry when box == the index set's ghost box,
//   * the X-only overloads (:3110-3139): markers whose getCellIndex cell is in box,
//   * the per-axis frame shift of side/node/edge data (:1017-1053), which the
//     C-ABI applies for the SIDE/NODE/EDGE centerings.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <mutex>
#include <string>

#include "../../include/ibtk_le.h"
#include "../../include/ibtk_le/LEInteractor.h"

namespace IBTK {
namespace {

struct Facade {
    std::mutex mu;
    int device = 0;
    void* stream = nullptr;
    ibtk_le_ctx ctx = nullptr;
    ibtk_le_markers m = nullptr;
    int* filt_idx = nullptr;
    double* filt_xs = nullptr;
    size_t filt_cap = 0;
    void ensure() {
        if (ctx) return;
        check(ibtk_le_ctx_create(device, stream, &ctx));
        check(ibtk_le_markers_create(ctx, &m));
    }
    static void check(int rc) {
        if (rc != IBTK_LE_OK) throw LEInteractorError(rc, ibtk_le_last_error());
    }
    void ensure_filter(size_t n, int ndim) {
        if (n <= filt_cap) return;
        if (filt_idx) hipFree(filt_idx);
        if (filt_xs) hipFree(filt_xs);
        filt_idx = nullptr;
        filt_xs = nullptr;
        if (hipMalloc(&filt_idx, sizeof(int) * n) != hipSuccess ||
            hipMalloc(&filt_xs, sizeof(double) * n * ndim) != hipSuccess)
            throw LEInteractorError(IBTK_LE_ERR_NOMEM, "LEInteractor: device allocation failed");
        filt_cap = n;
    }
};

Facade& F() {
    static Facade f;
    return f;
}

int kernel_of(const std::string& name) {
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

struct List {
    const int* idx;
    const double* xs;
    int n;
};

// LEInteractor::buildLocalIndices (LEInteractor.cpp:3031-3108)
List select_list(const LIndexSetView& idx, const PatchView& patch, const Box& box) {
    if (box == patch.box) return {idx.interior_local_indices, idx.interior_periodic_shifts, idx.n_interior};
    if (box == idx.ghost_box) return {idx.local_indices, idx.periodic_shifts, idx.n};
    throw LEInteractorError(IBTK_LE_ERR_ARG,
                            "LEInteractor: index-set overloads support box == patch box (interior nodes) or box == "
                            "the index set's ghost box (all nodes); other boxes need the per-cell node sets");
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

void do_interp(int centering, double* const* arrays, int q_depth, const int* ghost, LDataView Q, const double* X,
               const List& list, const PatchView& patch, const std::string& fcn) {
    const int k = kernel_of(fcn);
    Facade& f = F();
    std::lock_guard<std::mutex> lock(f.mu);
    f.ensure();
    const ibtk_le_patch_geom g = make_geom(patch, ghost);
    const int gmin = min_ghost(ghost, g.ndim);
    if (gmin < ibtk_le_min_ghost_width(k))
        throw LEInteractorError(IBTK_LE_ERR_GHOST_WIDTH,
                                "LEInteractor::interpolate(): insufficient ghost cells:  kernel function = " + fcn);
    if (list.n == 0) return;
    Facade::check(ibtk_le_markers_bin(f.ctx, f.m, &g, k, X, list.idx, list.xs, list.n));
    Facade::check(ibtk_le_interp(f.ctx, f.m, k, centering, 0, &g, arrays, q_depth, Q.ptr, Q.depth, X));
}

void do_spread(int centering, double* const* arrays, int q_depth, const int* ghost, const double* Q, int Q_depth,
               const double* X, const List& list, const PatchView& patch, const std::string& fcn) {
    const int k = kernel_of(fcn);
    Facade& f = F();
    std::lock_guard<std::mutex> lock(f.mu);
    f.ensure();
    const ibtk_le_patch_geom g = make_geom(patch, ghost);
    if (touches_physical(patch) && min_ghost(ghost, g.ndim) < ibtk_le_min_ghost_width(k))
        throw LEInteractorError(IBTK_LE_ERR_GHOST_WIDTH,
                                "LEInteractor::spread(): insufficient ghost cells at physical boundary:  kernel "
                                "function = " + fcn);
    if (list.n == 0) return;
    Facade::check(ibtk_le_markers_bin(f.ctx, f.m, &g, k, X, list.idx, list.xs, list.n));
    Facade::check(ibtk_le_spread(f.ctx, f.m, k, centering, 0, &g, arrays, q_depth, Q, Q_depth, X));
}

void require_vector(const SideDataView& q, int Q_depth, const char* who) {
    if (Q_depth != q.box.ndim || q.depth != 1)
        throw LEInteractorError(IBTK_LE_ERR_DEPTH, std::string("LEInteractor::") + who +
                                                       "():\n  side-centered " + who +
                                                       " requires vector-valued data.\n");
}

}  // namespace

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

// ---- cell ----------------------------------------------------------------------
void LEInteractor::interpolate(LDataView Q, LDataView X, const LIndexSetView& idx, const CellDataView& q,
                               const PatchView& patch, const Box& box, const int*, const std::string& fcn) {
    double* arr[1] = {q.ptr};
    if (Q.depth != q.depth) throw LEInteractorError(IBTK_LE_ERR_DEPTH, "LEInteractor::interpolate(): Q depth != q depth");
    do_interp(IBTK_LE_CELL, arr, q.depth, q.ghost, Q, X.ptr, select_list(idx, patch, box), patch, fcn);
}
void LEInteractor::spread(const CellDataView& q, LDataView Q, LDataView X, const LIndexSetView& idx,
                          const PatchView& patch, const Box& box, const int*, const std::string& fcn) {
    double* arr[1] = {q.ptr};
    if (Q.depth != q.depth) throw LEInteractorError(IBTK_LE_ERR_DEPTH, "LEInteractor::spread(): Q depth != q depth");
    do_spread(IBTK_LE_CELL, arr, q.depth, q.ghost, Q.ptr, Q.depth, X.ptr, select_list(idx, patch, box), patch, fcn);
}
// ---- node ----------------------------------------------------------------------
void LEInteractor::interpolateNode(LDataView Q, LDataView X, const LIndexSetView& idx, const NodeDataView& q,
                                   const PatchView& patch, const Box& box, const int*, const std::string& fcn) {
    double* arr[1] = {q.ptr};
    if (Q.depth != q.depth) throw LEInteractorError(IBTK_LE_ERR_DEPTH, "LEInteractor::interpolate(): Q depth != q depth");
    do_interp(IBTK_LE_NODE, arr, q.depth, q.ghost, Q, X.ptr, select_list(idx, patch, box), patch, fcn);
}
void LEInteractor::spreadNode(const NodeDataView& q, LDataView Q, LDataView X, const LIndexSetView& idx,
                              const PatchView& patch, const Box& box, const int*, const std::string& fcn) {
    double* arr[1] = {q.ptr};
    if (Q.depth != q.depth) throw LEInteractorError(IBTK_LE_ERR_DEPTH, "LEInteractor::spread(): Q depth != q depth");
    do_spread(IBTK_LE_NODE, arr, q.depth, q.ghost, Q.ptr, Q.depth, X.ptr, select_list(idx, patch, box), patch, fcn);
}
// ---- side ----------------------------------------------------------------------
void LEInteractor::interpolate(LDataView Q, LDataView X, const LIndexSetView& idx, const SideDataView& q,
                               const PatchView& patch, const Box& box, const int*, const std::string& fcn) {
    require_vector(q, Q.depth, "interpolate");
    do_interp(IBTK_LE_SIDE, const_cast<double* const*>(q.ptr), 1, q.ghost, Q, X.ptr, select_list(idx, patch, box),
              patch, fcn);
}
void LEInteractor::spread(const SideDataView& q, LDataView Q, LDataView X, const LIndexSetView& idx,
                          const PatchView& patch, const Box& box, const int*, const std::string& fcn) {
    require_vector(q, Q.depth, "spread");
    do_spread(IBTK_LE_SIDE, const_cast<double* const*>(q.ptr), 1, q.ghost, Q.ptr, Q.depth, X.ptr,
              select_list(idx, patch, box), patch, fcn);
}
// ---- edge (3-D) ------------------------------------------------------------------
void LEInteractor::interpolateEdge(LDataView Q, LDataView X, const LIndexSetView& idx, const EdgeDataView& q,
                                   const PatchView& patch, const Box& box, const int*, const std::string& fcn) {
    require_vector(q, Q.depth, "interpolate");
    do_interp(IBTK_LE_EDGE, const_cast<double* const*>(q.ptr), 1, q.ghost, Q, X.ptr, select_list(idx, patch, box),
              patch, fcn);
}
void LEInteractor::spreadEdge(const EdgeDataView& q, LDataView Q, LDataView X, const LIndexSetView& idx,
                              const PatchView& patch, const Box& box, const int*, const std::string& fcn) {
    require_vector(q, Q.depth, "spread");
    do_spread(IBTK_LE_EDGE, const_cast<double* const*>(q.ptr), 1, q.ghost, Q.ptr, Q.depth, X.ptr,
              select_list(idx, patch, box), patch, fcn);
}

// ---- X-only overloads (LEInteractor.cpp:3110-3139) ---------------------------------
static List filter_by_box(const PatchView& patch, const Box& box, const double* X, int X_size, int X_depth) {
    Facade& f = F();
    f.ensure();
    const int n = X_size / X_depth;
    const int zero[3] = {0, 0, 0};
    const ibtk_le_patch_geom g = make_geom(patch, zero);
    f.ensure_filter((size_t)std::max(n, 1), patch.box.ndim);
    int count = 0;
    Facade::check(ibtk_le_box_index_list(f.ctx, &g, X, n, box.lower, box.upper, f.filt_idx, (int)f.filt_cap, &count));
    return {f.filt_idx, nullptr, count};
}

void LEInteractor::interpolate(double* Q_data, int Q_depth, const double* X_data, int X_depth, int X_size,
                               const SideDataView& q, const PatchView& patch, const Box& box,
                               const std::string& fcn) {
    require_vector(q, Q_depth, "interpolate");
    List l;
    {
        std::lock_guard<std::mutex> lock(F().mu);
        l = filter_by_box(patch, box, X_data, X_size, X_depth);
    }
    LDataView Q{Q_data, Q_depth, X_size / X_depth};
    do_interp(IBTK_LE_SIDE, const_cast<double* const*>(q.ptr), 1, q.ghost, Q, X_data, l, patch, fcn);
}

void LEInteractor::spread(const SideDataView& q, const double* Q_data, int Q_depth, const double* X_data,
                          int X_depth, int X_size, const PatchView& patch, const Box& box, const std::string& fcn) {
    require_vector(q, Q_depth, "spread");
    List l;
    {
        std::lock_guard<std::mutex> lock(F().mu);
        l = filter_by_box(patch, box, X_data, X_size, X_depth);
    }
    do_spread(IBTK_LE_SIDE, const_cast<double* const*>(q.ptr), 1, q.ghost, Q_data, Q_depth, X_data, l, patch, fcn);
}

}  // namespace IBTK
