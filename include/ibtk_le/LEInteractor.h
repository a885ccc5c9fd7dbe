// LEInteractor.h -- C++ facade of IBTK::LEInteractor over the MI355X kernels.
//
// Mirrors the static interface of ibtk/include/ibtk/LEInteractor.h:100-993:
// getStencilSize, getMinimumGhostWidth, and the 32 interpolate / spread
// overloads -- on Cell / Node / Side / Edge data (overloaded by data type, as in
// the reference), in four argument forms each:
//   (a) LData Q and X with an index set, a box and a periodic shift
//       (LEInteractor.h:146-224, 459-566);
//   (b) raw Q / X arrays with an index set (:226-300, 571-684);
//   (c) std::vector<double> Q / X, the markers whose cell lies in the box
//       (:302-346, 690-796);
//   (d) raw Q / X arrays with their sizes, likewise (:348-455, 798-993).
// SAMRAI and PETSc are not part of this build, so their objects are replaced by
// light views carrying exactly what the reference reads from them: the patch box
// and Cartesian geometry (CartesianPatchGeometry), the ghosted arrays and their
// boxes (pdat::*Data), the marker arrays (LData's ghosted Vec array) and the
// cached index lists of LIndexSetData (LIndexSetData.cpp:83-169).
//
// Memory: the LData views, the raw-array overloads (b, d) and the data views
// hold DEVICE pointers.  The std::vector overloads (c) take HOST vectors, as the
// reference's do: X and Q are staged to the device and the interpolated Q is
// copied back before the call returns.
//
// Errors: the reference aborts through TBOX_ERROR; the facade throws
// IBTK::LEInteractorError carrying the same message and an IBTK_LE_ERR_* code.
#pragma once

#include <ostream>
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

namespace detail {
// pdat::CellData / NodeData<NDIM,double>: one ghosted Fortran-ordered array of
// `depth` components (depth slowest).  The tag makes Cell and Node distinct types.
template <int TAG>
struct ScalarDataView {
    double* ptr = nullptr;
    Box box;  // patch box (getBox())
    int ghost[3] = {0, 0, 0};
    int depth = 1;
};
// pdat::SideData / EdgeData<NDIM,double>: NDIM ghosted arrays (getPointer(axis)).
template <int TAG>
struct VectorDataView {
    double* ptr[3] = {nullptr, nullptr, nullptr};
    Box box;
    int ghost[3] = {0, 0, 0};
    int depth = 1;
};
}  // namespace detail
using CellDataView = detail::ScalarDataView<0>;
using NodeDataView = detail::ScalarDataView<1>;
using SideDataView = detail::VectorDataView<0>;
using EdgeDataView = detail::VectorDataView<1>;

// LData: ghosted blocked Vec array, AoS [local + ghost][depth]
struct LDataView {
    double* ptr = nullptr;
    int depth = 3;
    int local_size = 0;  // number of local + ghost nodes
};

// LIndexSetData<T> cached lists (LIndexSetData.cpp:83-169), device arrays in
// the reference's order (ibtk_le_index_set_list / ibtk_le_index_set_box_list
// build them).  T is the node type of the reference's template (LNode or
// LNodeIndex); the lists are the same.  `cells` (NDIM ints per entry of the
// all-nodes list: the IndexData cell each node sits in) lets buildLocalIndices
// serve boxes other than the patch box and the ghost box (LEInteractor.cpp:
// 3070-3106); without it those boxes throw IBTK_LE_ERR_ARG.
struct LIndexSetBase {
    Box ghost_box;                       // idx_data->getGhostBox()
    const int* local_indices = nullptr;  // all nodes in the ghost box
    const double* periodic_shifts = nullptr;
    const int* cells = nullptr;          // the cell of each of those nodes (optional)
    int n = 0;
    const int* interior_local_indices = nullptr;  // nodes in the patch interior
    const double* interior_periodic_shifts = nullptr;
    int n_interior = 0;
};
struct LNode {};
struct LNodeIndex {};
template <class T = LNode>
struct LIndexSetDataView : LIndexSetBase {};
using LIndexSetView = LIndexSetDataView<LNode>;

class LEInteractor {
public:
    // The USER_DEFINED kernel function and its stencil size (LEInteractor.h:100-101):
    // read at every USER_DEFINED call.  Initially IB_4's kernel function
    // (ibtk_le_ib4_kernel_fcn = ib4_kernel_fcn, LEInteractor.cpp:629-651), as in the
    // reference; nullptr also means it.
    static double (*s_kernel_fcn)(double r);
    static int s_kernel_fcn_stencil_size;

    static void setFromDatabase(const void* db = nullptr);  // no settable data (LEInteractor.cpp:654-658)
    static void printClassData(std::ostream& os);
    static int getStencilSize(const std::string& kernel_fcn);
    static int getMinimumGhostWidth(const std::string& kernel_fcn);

    // (a) LData + index set (LEInteractor.h:146-224) ------------------------------
    static void interpolate(LDataView Q_data, LDataView X_data, const LIndexSetBase& idx_data,
                            const CellDataView& q_data, const PatchView& patch, const Box& interp_box,
                            const int* periodic_shift, const std::string& interp_fcn = "IB_4");
    static void interpolate(LDataView Q_data, LDataView X_data, const LIndexSetBase& idx_data,
                            const NodeDataView& q_data, const PatchView& patch, const Box& interp_box,
                            const int* periodic_shift, const std::string& interp_fcn = "IB_4");
    static void interpolate(LDataView Q_data, LDataView X_data, const LIndexSetBase& idx_data,
                            const SideDataView& q_data, const PatchView& patch, const Box& interp_box,
                            const int* periodic_shift, const std::string& interp_fcn = "IB_4");
    static void interpolate(LDataView Q_data, LDataView X_data, const LIndexSetBase& idx_data,
                            const EdgeDataView& q_data, const PatchView& patch, const Box& interp_box,
                            const int* periodic_shift, const std::string& interp_fcn = "IB_4");
    // (b) raw arrays + index set (:226-300) ---------------------------------------
    static void interpolate(double* Q_data, int Q_depth, const double* X_data, int X_depth,
                            const LIndexSetBase& idx_data, const CellDataView& q_data, const PatchView& patch,
                            const Box& interp_box, const int* periodic_shift,
                            const std::string& interp_fcn = "IB_4");
    static void interpolate(double* Q_data, int Q_depth, const double* X_data, int X_depth,
                            const LIndexSetBase& idx_data, const NodeDataView& q_data, const PatchView& patch,
                            const Box& interp_box, const int* periodic_shift,
                            const std::string& interp_fcn = "IB_4");
    static void interpolate(double* Q_data, int Q_depth, const double* X_data, int X_depth,
                            const LIndexSetBase& idx_data, const SideDataView& q_data, const PatchView& patch,
                            const Box& interp_box, const int* periodic_shift,
                            const std::string& interp_fcn = "IB_4");
    static void interpolate(double* Q_data, int Q_depth, const double* X_data, int X_depth,
                            const LIndexSetBase& idx_data, const EdgeDataView& q_data, const PatchView& patch,
                            const Box& interp_box, const int* periodic_shift,
                            const std::string& interp_fcn = "IB_4");
    // (c) host vectors, the markers whose cell lies in the box (:302-346) ----------
    static void interpolate(std::vector<double>& Q_data, int Q_depth, const std::vector<double>& X_data,
                            int X_depth, const CellDataView& q_data, const PatchView& patch, const Box& interp_box,
                            const std::string& interp_fcn = "IB_4");
    static void interpolate(std::vector<double>& Q_data, int Q_depth, const std::vector<double>& X_data,
                            int X_depth, const NodeDataView& q_data, const PatchView& patch, const Box& interp_box,
                            const std::string& interp_fcn = "IB_4");
    static void interpolate(std::vector<double>& Q_data, int Q_depth, const std::vector<double>& X_data,
                            int X_depth, const SideDataView& q_data, const PatchView& patch, const Box& interp_box,
                            const std::string& interp_fcn = "IB_4");
    static void interpolate(std::vector<double>& Q_data, int Q_depth, const std::vector<double>& X_data,
                            int X_depth, const EdgeDataView& q_data, const PatchView& patch, const Box& interp_box,
                            const std::string& interp_fcn = "IB_4");
    // (d) raw arrays with sizes, likewise (:348-455) --------------------------------
    static void interpolate(double* Q_data, int Q_size, int Q_depth, const double* X_data, int X_size, int X_depth,
                            const CellDataView& q_data, const PatchView& patch, const Box& interp_box,
                            const std::string& interp_fcn = "IB_4");
    static void interpolate(double* Q_data, int Q_size, int Q_depth, const double* X_data, int X_size, int X_depth,
                            const NodeDataView& q_data, const PatchView& patch, const Box& interp_box,
                            const std::string& interp_fcn = "IB_4");
    static void interpolate(double* Q_data, int Q_size, int Q_depth, const double* X_data, int X_size, int X_depth,
                            const SideDataView& q_data, const PatchView& patch, const Box& interp_box,
                            const std::string& interp_fcn = "IB_4");
    static void interpolate(double* Q_data, int Q_size, int Q_depth, const double* X_data, int X_size, int X_depth,
                            const EdgeDataView& q_data, const PatchView& patch, const Box& interp_box,
                            const std::string& interp_fcn = "IB_4");

    // (a) LData + index set (LEInteractor.h:459-566) ------------------------------
    static void spread(const CellDataView& q_data, LDataView Q_data, LDataView X_data,
                       const LIndexSetBase& idx_data, const PatchView& patch, const Box& spread_box,
                       const int* periodic_shift, const std::string& spread_fcn = "IB_4");
    static void spread(const NodeDataView& q_data, LDataView Q_data, LDataView X_data,
                       const LIndexSetBase& idx_data, const PatchView& patch, const Box& spread_box,
                       const int* periodic_shift, const std::string& spread_fcn = "IB_4");
    static void spread(const SideDataView& q_data, LDataView Q_data, LDataView X_data,
                       const LIndexSetBase& idx_data, const PatchView& patch, const Box& spread_box,
                       const int* periodic_shift, const std::string& spread_fcn = "IB_4");
    static void spread(const EdgeDataView& q_data, LDataView Q_data, LDataView X_data,
                       const LIndexSetBase& idx_data, const PatchView& patch, const Box& spread_box,
                       const int* periodic_shift, const std::string& spread_fcn = "IB_4");
    // (b) raw arrays + index set (:571-684) ---------------------------------------
    static void spread(const CellDataView& q_data, const double* Q_data, int Q_depth, const double* X_data,
                       int X_depth, const LIndexSetBase& idx_data, const PatchView& patch, const Box& spread_box,
                       const int* periodic_shift, const std::string& spread_fcn = "IB_4");
    static void spread(const NodeDataView& q_data, const double* Q_data, int Q_depth, const double* X_data,
                       int X_depth, const LIndexSetBase& idx_data, const PatchView& patch, const Box& spread_box,
                       const int* periodic_shift, const std::string& spread_fcn = "IB_4");
    static void spread(const SideDataView& q_data, const double* Q_data, int Q_depth, const double* X_data,
                       int X_depth, const LIndexSetBase& idx_data, const PatchView& patch, const Box& spread_box,
                       const int* periodic_shift, const std::string& spread_fcn = "IB_4");
    static void spread(const EdgeDataView& q_data, const double* Q_data, int Q_depth, const double* X_data,
                       int X_depth, const LIndexSetBase& idx_data, const PatchView& patch, const Box& spread_box,
                       const int* periodic_shift, const std::string& spread_fcn = "IB_4");
    // (c) host vectors (:690-796) ----------------------------------------------------
    static void spread(const CellDataView& q_data, const std::vector<double>& Q_data, int Q_depth,
                       const std::vector<double>& X_data, int X_depth, const PatchView& patch,
                       const Box& spread_box, const std::string& spread_fcn = "IB_4");
    static void spread(const NodeDataView& q_data, const std::vector<double>& Q_data, int Q_depth,
                       const std::vector<double>& X_data, int X_depth, const PatchView& patch,
                       const Box& spread_box, const std::string& spread_fcn = "IB_4");
    static void spread(const SideDataView& q_data, const std::vector<double>& Q_data, int Q_depth,
                       const std::vector<double>& X_data, int X_depth, const PatchView& patch,
                       const Box& spread_box, const std::string& spread_fcn = "IB_4");
    static void spread(const EdgeDataView& q_data, const std::vector<double>& Q_data, int Q_depth,
                       const std::vector<double>& X_data, int X_depth, const PatchView& patch,
                       const Box& spread_box, const std::string& spread_fcn = "IB_4");
    // (d) raw arrays with sizes (:798-993) -------------------------------------------
    static void spread(const CellDataView& q_data, const double* Q_data, int Q_size, int Q_depth,
                       const double* X_data, int X_size, int X_depth, const PatchView& patch,
                       const Box& spread_box, const std::string& spread_fcn = "IB_4");
    static void spread(const NodeDataView& q_data, const double* Q_data, int Q_size, int Q_depth,
                       const double* X_data, int X_size, int X_depth, const PatchView& patch,
                       const Box& spread_box, const std::string& spread_fcn = "IB_4");
    static void spread(const SideDataView& q_data, const double* Q_data, int Q_size, int Q_depth,
                       const double* X_data, int X_size, int X_depth, const PatchView& patch,
                       const Box& spread_box, const std::string& spread_fcn = "IB_4");
    static void spread(const EdgeDataView& q_data, const double* Q_data, int Q_size, int Q_depth,
                       const double* X_data, int X_size, int X_depth, const PatchView& patch,
                       const Box& spread_box, const std::string& spread_fcn = "IB_4");

    // Stream / device of the facade's context (default: device 0, null stream).
    static void setStream(int device, void* hip_stream);
    static void synchronize();
};

}  // namespace IBTK
