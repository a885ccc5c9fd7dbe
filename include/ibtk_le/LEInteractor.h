// LEInteractor.h -- C++ facade of IBTK::LEInteractor over the MI355X kernels.
//
// Mirrors the static interface of ibtk/include/ibtk/LEInteractor.h:100-993
// (getStencilSize, getMinimumGhostWidth, interpolate/spread on Cell/Node/Side/
// Edge data with an index set, a patch, a box, a periodic shift and the kernel
// string; the raw double* overloads; the X-only overloads without index sets).
// SAMRAI and PETSc are not part of this build, so the SAMRAI/PETSc objects are
// replaced by light views that carry exactly what the reference reads from
// them: the patch box and Cartesian geometry (CartesianPatchGeometry), the
// ghosted arrays and their boxes (pdat::*Data), the marker arrays (LData's
// ghosted Vec array) and the cached index lists of LIndexSetData
// (LIndexSetData.cpp:83-169).  Every data pointer is a DEVICE pointer.
//
// Errors: the reference aborts through TBOX_ERROR; the facade throws
// IBTK::LEInteractorError carrying the same message.
#pragma once

#include <stdexcept>
#include <string>
#include <vector>

#include "../ibtk_le.h"

namespace IBTK {

struct LEInteractorError : public std::runtime_error {
    int code;
    LEInteractorError(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

// hier::Box<NDIM> (inclusive bounds)
struct Box {
    int ndim = 3;
    int lower[3] = {0, 0, 0};
    int upper[3] = {-1, -1, -1};
    bool operator==(const Box& o) const {
        if (ndim != o.ndim) return false;
        for (int d = 0; d < ndim; ++d)
            if (lower[d] != o.lower[d] || upper[d] != o.upper[d]) return false;
        return true;
    }
    Box grow(int g) const {
        Box b = *this;
        for (int d = 0; d < ndim; ++d) {
            b.lower[d] -= g;
            b.upper[d] += g;
        }
        return b;
    }
};

// hier::Patch + geom::CartesianPatchGeometry
struct PatchView {
    Box box;
    double dx[3] = {1, 1, 1};
    double x_lower[3] = {0, 0, 0};
    double x_upper[3] = {1, 1, 1};
    bool touches_physical_bdry[3][2] = {{false, false}, {false, false}, {false, false}};  // getTouchesRegularBoundary
};

// pdat::{Cell,Node,Side,Edge}Data<NDIM,double>: ghosted Fortran-ordered arrays
struct CellDataView {
    double* ptr = nullptr;  // depth arrays, depth slowest
    Box box;                // patch box (getBox())
    int ghost[3] = {0, 0, 0};
    int depth = 1;
};
using NodeDataView = CellDataView;
struct SideDataView {
    double* ptr[3] = {nullptr, nullptr, nullptr};  // getPointer(axis)
    Box box;
    int ghost[3] = {0, 0, 0};
    int depth = 1;
};
using EdgeDataView = SideDataView;

// LData: ghosted blocked Vec array, AoS [local + ghost][depth]
struct LDataView {
    double* ptr = nullptr;
    int depth = 3;
    int local_size = 0;  // number of local + ghost nodes
};

// LIndexSetData cached lists (LIndexSetData.cpp:83-169), device arrays
struct LIndexSetView {
    Box ghost_box;                       // idx_data->getGhostBox()
    const int* local_indices = nullptr;  // all nodes in the ghost box
    const double* periodic_shifts = nullptr;
    int n = 0;
    const int* interior_local_indices = nullptr;  // nodes in the patch interior
    const double* interior_periodic_shifts = nullptr;
    int n_interior = 0;
};

class LEInteractor {
public:
    static int getStencilSize(const std::string& kernel_fcn);
    static int getMinimumGhostWidth(const std::string& kernel_fcn);

    // --- index-set overloads (LEInteractor.h:146-330, 557-760) -------------------
    static void interpolate(LDataView Q_data, LDataView X_data, const LIndexSetView& idx_data,
                            const CellDataView& q_data, const PatchView& patch, const Box& interp_box,
                            const int* periodic_shift, const std::string& interp_fcn = "IB_4");
    static void interpolate(LDataView Q_data, LDataView X_data, const LIndexSetView& idx_data,
                            const SideDataView& q_data, const PatchView& patch, const Box& interp_box,
                            const int* periodic_shift, const std::string& interp_fcn = "IB_4");
    static void interpolateNode(LDataView Q_data, LDataView X_data, const LIndexSetView& idx_data,
                                const NodeDataView& q_data, const PatchView& patch, const Box& interp_box,
                                const int* periodic_shift, const std::string& interp_fcn = "IB_4");
    static void interpolateEdge(LDataView Q_data, LDataView X_data, const LIndexSetView& idx_data,
                                const EdgeDataView& q_data, const PatchView& patch, const Box& interp_box,
                                const int* periodic_shift, const std::string& interp_fcn = "IB_4");

    static void spread(const CellDataView& q_data, LDataView Q_data, LDataView X_data,
                       const LIndexSetView& idx_data, const PatchView& patch, const Box& spread_box,
                       const int* periodic_shift, const std::string& spread_fcn = "IB_4");
    static void spread(const SideDataView& q_data, LDataView Q_data, LDataView X_data,
                       const LIndexSetView& idx_data, const PatchView& patch, const Box& spread_box,
                       const int* periodic_shift, const std::string& spread_fcn = "IB_4");
    static void spreadNode(const NodeDataView& q_data, LDataView Q_data, LDataView X_data,
                           const LIndexSetView& idx_data, const PatchView& patch, const Box& spread_box,
                           const int* periodic_shift, const std::string& spread_fcn = "IB_4");
    static void spreadEdge(const EdgeDataView& q_data, LDataView Q_data, LDataView X_data,
                           const LIndexSetView& idx_data, const PatchView& patch, const Box& spread_box,
                           const int* periodic_shift, const std::string& spread_fcn = "IB_4");

    // --- X-only overloads without index sets (LEInteractor.cpp:3110-3139):
    // every marker whose cell (IndexUtilities::getCellIndex) lies in `box`, no
    // periodic shifts.  X_size is the number of doubles in X (nodes * NDIM).
    static void interpolate(double* Q_data, int Q_depth, const double* X_data, int X_depth, int X_size,
                            const SideDataView& q_data, const PatchView& patch, const Box& interp_box,
                            const std::string& interp_fcn = "IB_4");
    static void spread(const SideDataView& q_data, const double* Q_data, int Q_depth, const double* X_data,
                       int X_depth, int X_size, const PatchView& patch, const Box& spread_box,
                       const std::string& spread_fcn = "IB_4");

    // Stream / device of the facade's context (default: device 0, null stream).
    static void setStream(int device, void* hip_stream);
    static void synchronize();
};

}  // namespace IBTK
