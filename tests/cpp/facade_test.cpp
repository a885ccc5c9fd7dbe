// facade_test.cpp -- drives every overload form of the IBTK::LEInteractor C++ facade
// (include/ibtk_le/LEInteractor.h) on the GPU, the way LDataManager drives
// LEInteractor (LDataManager.cpp:625-660, 763-807), for Cell / Node / Side / Edge
// data on one periodic 3-D patch.  tests/test_gpu_boundary.py::test_cpp_facade
// writes the inputs (markers, fields, the index set's lists made by the oracle)
// into a directory, runs this program on it and compares what it writes back
// with the oracle.  Forms (LEInteractor.h:146-993):
//   a  LData views + index set      (interior list for interp, ghost list for spread)
//   b  raw device arrays + index set (same lists: must equal a bit for bit)
//   c  host std::vector, box filter  (markers whose cell is in a sub-box, no shifts)
//   d  raw device arrays with sizes, box filter (must equal c bit for bit)
//   u  USER_DEFINED (LEInteractor::s_kernel_fcn), form a's lists
//   e  LData views + index set over a sub-box reaching into the ghost cells
//      (buildLocalIndices' box branch, LEInteractor.cpp:3070-3106, through the
//      index set's cells)
// Then a patch with physical faces: the spread ghost-width check
// (LEInteractor.cpp:2729-2745) and the spread + physical-boundary fold of
// LDataManager::spread (LDataManager.cpp:625-659) on side data.
// Prints "FACADE OK" after the error-convention checks.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <string>
#include <type_traits>
#include <vector>

#include "ibtk_le.h"
#include "ibtk_le/LEInteractor.h"

using namespace IBTK;

#define HC(x)                                                                  \
    do {                                                                       \
        if ((x) != hipSuccess) {                                               \
            std::printf("hip failure %s\n", #x);                               \
            std::exit(1);                                                      \
        }                                                                      \
    } while (0)
#define EXPECT(c, msg)                                                         \
    do {                                                                       \
        if (!(c)) {                                                            \
            std::printf("FAIL: %s\n", msg);                                    \
            std::exit(1);                                                      \
        }                                                                      \
    } while (0)

static std::string D;

template <class T>
static std::vector<T> load(const std::string& name, size_t n) {
    std::vector<T> v(n);
    FILE* f = std::fopen((D + "/" + name).c_str(), "rb");
    EXPECT(f, ("open " + name).c_str());
    EXPECT(std::fread(v.data(), sizeof(T), n, f) == n, ("read " + name).c_str());
    std::fclose(f);
    return v;
}
template <class T>
static void save(const std::string& name, const T* p, size_t n) {
    FILE* f = std::fopen((D + "/" + name).c_str(), "wb");
    EXPECT(f && std::fwrite(p, sizeof(T), n, f) == n, ("write " + name).c_str());
    std::fclose(f);
}
template <class T>
static T* upload(const std::vector<T>& h) {
    T* d = nullptr;
    HC(hipMalloc(&d, sizeof(T) * (h.size() ? h.size() : 1)));
    if (!h.empty()) HC(hipMemcpy(d, h.data(), sizeof(T) * h.size(), hipMemcpyHostToDevice));
    return d;
}
static std::vector<double> download(const double* d, size_t n) {
    std::vector<double> h(n);
    HC(hipMemcpy(h.data(), d, sizeof(double) * n, hipMemcpyDeviceToHost));
    return h;
}

int N, g, M, n_int, n_all, depth_c;
Box sub;  // the sub-box of forms c, d, e
PatchView patch;
LIndexSetView idx;
double *Xd, *Fd;
std::vector<double> hX, hF;
const int pshift[3] = {0, 0, 0};

// array size of component a of a centering (ghosted), elements
static size_t asize(const char* c, int a, int depth) {
    size_t n = (size_t)depth;
    for (int d = 0; d < 3; ++d) {
        int e = N + 2 * g;
        if (c[0] == 'n') e += 1;
        if (c[0] == 's' && d == a) e += 1;
        if (c[0] == 'e' && d != a) e += 1;
        n *= (size_t)e;
    }
    return n;
}

// the four forms of interp and spread on one data view type
// the USER_DEFINED form's kernel function: (9/4 - r^2)/4 inside |r| < 3/2 (+ and * only,
// as tests/test_gpu_boundary.py evaluates it for the oracle)
static double user_phi3(double r) {
    const double r2 = r * r;
    return r2 < 2.25 ? (2.25 - r2) * 0.25 : 0.0;
}

template <class V>
static void run(const char* cname, V& u, V& f, int ncomp, int depth, int Qdepth) {
    auto fptr = [&](int a) -> double*& {
        if constexpr (std::is_same_v<V, CellDataView> || std::is_same_v<V, NodeDataView>) return f.ptr;
        else return f.ptr[a];
    };
    auto zero_f = [&]() {
        for (int a = 0; a < ncomp; ++a) HC(hipMemset(fptr(a), 0, sizeof(double) * asize(cname, a, depth)));
    };
    auto save_f = [&](const std::string& form) {
        for (int a = 0; a < ncomp; ++a) {
            auto h = download(fptr(a), asize(cname, a, depth));
            save(std::string("f_") + cname + "_" + form + "_" + std::to_string(a) + ".bin", h.data(), h.size());
        }
    };
    const size_t nQ = (size_t)M * Qdepth;
    std::vector<double> init(nQ, -7.0);
    double* Qd = upload(init);
    std::vector<double> hQ2(3 * (size_t)M);
    for (int s = 0; s < M; ++s)
        for (int k = 0; k < Qdepth; ++k) hQ2[(size_t)s * Qdepth + k] = hF[3 * (size_t)s + (k % 3)];
    hQ2.resize(nQ);
    double* Sd = upload(hQ2);  // the spread values, depth Qdepth
    LDataView Qv{Qd, Qdepth, M}, Xv{Xd, 3, M}, Sv{Sd, Qdepth, M};
    const Box ghost_box = idx.ghost_box;
    // a: LData + index set
    LEInteractor::interpolate(Qv, Xv, idx, u, patch, patch.box, pshift, "IB_4");
    LEInteractor::synchronize();
    auto h = download(Qd, nQ);
    save(std::string("Q_") + cname + "_a.bin", h.data(), nQ);
    zero_f();
    LEInteractor::spread(f, Sv, Xv, idx, patch, ghost_box, pshift, "IB_4");
    LEInteractor::synchronize();
    save_f("a");
    // b: raw arrays + index set
    HC(hipMemcpy(Qd, init.data(), sizeof(double) * nQ, hipMemcpyHostToDevice));
    LEInteractor::interpolate(Qd, Qdepth, Xd, 3, idx, u, patch, patch.box, pshift, "IB_4");
    LEInteractor::synchronize();
    h = download(Qd, nQ);
    save(std::string("Q_") + cname + "_b.bin", h.data(), nQ);
    zero_f();
    LEInteractor::spread(f, Sd, Qdepth, Xd, 3, idx, patch, ghost_box, pshift, "IB_4");
    LEInteractor::synchronize();
    save_f("b");
    // c: host vectors, the markers whose cell is in the sub-box
    std::vector<double> Qh(init);
    LEInteractor::interpolate(Qh, Qdepth, hX, 3, u, patch, sub, "IB_4");
    save(std::string("Q_") + cname + "_c.bin", Qh.data(), nQ);
    zero_f();
    LEInteractor::spread(f, hQ2, Qdepth, hX, 3, patch, sub, "IB_4");
    LEInteractor::synchronize();
    save_f("c");
    // d: raw arrays with sizes
    HC(hipMemcpy(Qd, init.data(), sizeof(double) * nQ, hipMemcpyHostToDevice));
    LEInteractor::interpolate(Qd, (int)nQ, Qdepth, Xd, 3 * M, 3, u, patch, sub, "IB_4");
    LEInteractor::synchronize();
    h = download(Qd, nQ);
    save(std::string("Q_") + cname + "_d.bin", h.data(), nQ);
    zero_f();
    LEInteractor::spread(f, Sd, (int)nQ, Qdepth, Xd, 3 * M, 3, patch, sub, "IB_4");
    LEInteractor::synchronize();
    save_f("d");
    // e: LData + index set over the sub-box
    HC(hipMemcpy(Qd, init.data(), sizeof(double) * nQ, hipMemcpyHostToDevice));
    LEInteractor::interpolate(Qv, Xv, idx, u, patch, sub, pshift, "IB_4");
    LEInteractor::synchronize();
    h = download(Qd, nQ);
    save(std::string("Q_") + cname + "_e.bin", h.data(), nQ);
    zero_f();
    LEInteractor::spread(f, Sv, Xv, idx, patch, sub, pshift, "IB_4");
    LEInteractor::synchronize();
    save_f("e");
    // u: USER_DEFINED through LEInteractor::s_kernel_fcn (a 3-point kernel function,
    // LEInteractor.cpp:2688, 3007), on form a's lists
    LEInteractor::s_kernel_fcn = &user_phi3;
    LEInteractor::s_kernel_fcn_stencil_size = 3;
    HC(hipMemcpy(Qd, init.data(), sizeof(double) * nQ, hipMemcpyHostToDevice));
    LEInteractor::interpolate(Qv, Xv, idx, u, patch, patch.box, pshift, "USER_DEFINED");
    LEInteractor::synchronize();
    h = download(Qd, nQ);
    save(std::string("Q_") + cname + "_u.bin", h.data(), nQ);
    zero_f();
    LEInteractor::spread(f, Sv, Xv, idx, patch, ghost_box, pshift, "USER_DEFINED");
    LEInteractor::synchronize();
    save_f("u");
    LEInteractor::s_kernel_fcn = &ibtk_le_ib4_kernel_fcn;  // the reference's default again
    LEInteractor::s_kernel_fcn_stencil_size = 4;
    HC(hipFree(Qd));
    HC(hipFree(Sd));
}

int main(int argc, char** argv) {
    EXPECT(argc == 2, "usage: facade_test <dir>");
    // the reference's initial s_kernel_fcn is ib4_kernel_fcn (LEInteractor.cpp:651)
    EXPECT(LEInteractor::s_kernel_fcn == &ibtk_le_ib4_kernel_fcn && LEInteractor::s_kernel_fcn_stencil_size == 4,
           "initial s_kernel_fcn");
    EXPECT(LEInteractor::s_kernel_fcn(0.0) == 0.5, "ib4_kernel_fcn(0)");
    D = argv[1];
    FILE* mf = std::fopen((D + "/meta.txt").c_str(), "r");
    EXPECT(mf && std::fscanf(mf, "%d %d %d %d %d %d", &N, &g, &M, &n_int, &n_all, &depth_c) == 6, "meta");
    sub.ndim = 3;
    EXPECT(std::fscanf(mf, "%d %d %d %d %d %d", &sub.lower[0], &sub.lower[1], &sub.lower[2], &sub.upper[0],
                       &sub.upper[1], &sub.upper[2]) == 6, "meta sub-box");
    std::fclose(mf);
    patch.box.ndim = 3;
    for (int d = 0; d < 3; ++d) {
        patch.box.lower[d] = 0;
        patch.box.upper[d] = N - 1;
        patch.dx[d] = 1.0 / N;
        patch.x_lower[d] = 0.0;
        patch.x_upper[d] = 1.0;
    }
    hX = load<double>("X.bin", 3 * (size_t)M);
    hF = load<double>("F.bin", 3 * (size_t)M);
    Xd = upload(hX);
    Fd = upload(hF);
    idx.ghost_box = patch.box.grow(g);
    idx.interior_local_indices = upload(load<int>("idx_int.bin", n_int));
    idx.interior_periodic_shifts = upload(load<double>("xs_int.bin", 3 * (size_t)n_int));
    idx.n_interior = n_int;
    idx.local_indices = upload(load<int>("idx_all.bin", n_all));
    idx.periodic_shifts = upload(load<double>("xs_all.bin", 3 * (size_t)n_all));
    idx.cells = upload(load<int>("cells_all.bin", 3 * (size_t)n_all));
    idx.n = n_all;

    EXPECT(LEInteractor::getStencilSize("IB_4") == 4 && LEInteractor::getMinimumGhostWidth("IB_6") == 4, "stencil");

    CellDataView uc, fc;
    uc.box = fc.box = patch.box;
    uc.depth = fc.depth = depth_c;
    NodeDataView un, fn;
    un.box = fn.box = patch.box;
    SideDataView us, fs;
    us.box = fs.box = patch.box;
    EdgeDataView ue, fe;
    ue.box = fe.box = patch.box;
    for (int d = 0; d < 3; ++d) uc.ghost[d] = fc.ghost[d] = un.ghost[d] = fn.ghost[d] = us.ghost[d] = fs.ghost[d] =
        ue.ghost[d] = fe.ghost[d] = g;
    uc.ptr = upload(load<double>("u_cell.bin", asize("cell", 0, depth_c)));
    HC(hipMalloc(&fc.ptr, sizeof(double) * asize("cell", 0, depth_c)));
    un.ptr = upload(load<double>("u_node.bin", asize("node", 0, 1)));
    HC(hipMalloc(&fn.ptr, sizeof(double) * asize("node", 0, 1)));
    for (int a = 0; a < 3; ++a) {
        us.ptr[a] = upload(load<double>("u_side" + std::to_string(a) + ".bin", asize("side", a, 1)));
        HC(hipMalloc(&fs.ptr[a], sizeof(double) * asize("side", a, 1)));
        ue.ptr[a] = upload(load<double>("u_edge" + std::to_string(a) + ".bin", asize("edge", a, 1)));
        HC(hipMalloc(&fe.ptr[a], sizeof(double) * asize("edge", a, 1)));
    }
    run("cell", uc, fc, 1, depth_c, depth_c);
    run("node", un, fn, 1, 1, 1);
    run("side", us, fs, 3, 1, 3);
    run("edge", ue, fe, 3, 1, 3);

    // error conventions (TBOX_ERROR -> LEInteractorError with an IBTK_LE_ERR_* code)
    double* Qd;
    HC(hipMalloc(&Qd, 24 * (size_t)M));
    LDataView Qv{Qd, 3, M}, Xv{Xd, 3, M};
    bool thrown = false;
    try {
        LEInteractor::interpolate(Qv, Xv, idx, us, patch, patch.box, pshift, "NOT_A_KERNEL");
    } catch (const LEInteractorError& e) {
        thrown = e.code == IBTK_LE_ERR_UNKNOWN_KERNEL;
    }
    EXPECT(thrown, "unknown kernel throws");
    thrown = false;
    try {
        LEInteractor::interpolate(Qv, Xv, idx, us, patch, patch.box, pshift, "IB_6");  // needs 4 ghosts
    } catch (const LEInteractorError& e) {
        thrown = e.code == IBTK_LE_ERR_GHOST_WIDTH;
    }
    EXPECT(thrown, "ghost width throws");
    thrown = false;
    try {
        LDataView Q2{Qd, 2, M};
        LEInteractor::interpolate(Q2, Xv, idx, us, patch, patch.box, pshift, "IB_4");
    } catch (const LEInteractorError& e) {
        thrown = e.code == IBTK_LE_ERR_DEPTH;
    }
    EXPECT(thrown, "side depth mismatch throws");
    thrown = false;
    try {
        LDataView Q2{Qd, 2, M};
        LEInteractor::spread(fe, Q2, Xv, idx, patch, idx.ghost_box, pshift, "IB_4");
    } catch (const LEInteractorError& e) {
        thrown = e.code == IBTK_LE_ERR_DEPTH;
    }
    EXPECT(thrown, "edge depth mismatch throws");
    thrown = false;
    try {
        LIndexSetView nocells = idx;
        nocells.cells = nullptr;
        LEInteractor::interpolate(Qv, Xv, nocells, us, patch, sub, pshift, "IB_4");
    } catch (const LEInteractorError& e) {
        thrown = e.code == IBTK_LE_ERR_ARG;
    }
    EXPECT(thrown, "a sub-box without the index set's cells throws");

    // a patch with physical faces in x and z, periodic in y (LEInteractor.cpp:2729-2745:
    // spreading near a physical boundary needs the ghost width; the fold follows, as
    // LDataManager::spread calls accumulateFromPhysicalBoundaryData), with its own
    // index set (no images across the physical faces)
    PatchView phys = patch;
    phys.touches_physical_bdry[0][0] = phys.touches_physical_bdry[0][1] = true;
    phys.touches_physical_bdry[2][0] = phys.touches_physical_bdry[2][1] = true;
    int n_phys = 0;
    {
        FILE* pf = std::fopen((D + "/meta_phys.txt").c_str(), "r");
        EXPECT(pf && std::fscanf(pf, "%d", &n_phys) == 1, "meta_phys");
        std::fclose(pf);
    }
    LIndexSetView idxp;
    idxp.ghost_box = patch.box.grow(g);
    idxp.local_indices = upload(load<int>("idx_phys.bin", n_phys));
    idxp.periodic_shifts = upload(load<double>("xs_phys.bin", 3 * (size_t)n_phys));
    idxp.n = n_phys;
    SideDataView fs1 = fs;
    for (int d = 0; d < 3; ++d) fs1.ghost[d] = 1;  // below IB_4's 3
    thrown = false;
    try {
        LEInteractor::spread(fs1, Qv, Xv, idxp, phys, idxp.ghost_box, pshift, "IB_4");
    } catch (const LEInteractorError& e) {
        thrown = e.code == IBTK_LE_ERR_GHOST_WIDTH;
    }
    EXPECT(thrown, "spread next to a physical boundary with too few ghosts throws");
    {
        std::vector<double> hS(3 * (size_t)M);
        for (size_t i = 0; i < hS.size(); ++i) hS[i] = hF[i];
        double* Sd = upload(hS);
        LDataView Sv{Sd, 3, M};
        for (int a = 0; a < 3; ++a) HC(hipMemset(fs.ptr[a], 0, sizeof(double) * asize("side", a, 1)));
        LEInteractor::spread(fs, Sv, Xv, idxp, phys, idxp.ghost_box, pshift, "IB_4");  // enough ghosts: no throw
        ibtk_le_patch_geom pg{};
        pg.ndim = 3;
        for (int d = 0; d < 3; ++d) {
            pg.ilower[d] = 0;
            pg.iupper[d] = N - 1;
            pg.gcw[d] = g;
            pg.dx[d] = 1.0 / N;
            pg.x_lower[d] = 0.0;
            pg.x_upper[d] = 1.0;
        }
        const int physf[6] = {1, 1, 0, 0, 1, 1};
        std::vector<double> ac = load<double>("bc_a.bin", 18), bc = load<double>("bc_b.bin", 18),
                            gc = load<double>("bc_g.bin", 18);
        ibtk_le_ctx c2 = nullptr;
        EXPECT(ibtk_le_ctx_create(0, nullptr, &c2) == IBTK_LE_OK, "ctx");
        double* arr[3] = {fs.ptr[0], fs.ptr[1], fs.ptr[2]};
        EXPECT(ibtk_le_phys_bdry_side(c2, &pg, arr, physf, ac.data(), bc.data(), gc.data(), 1) == IBTK_LE_OK, "fold");
        EXPECT(ibtk_le_ctx_synchronize(c2) == IBTK_LE_OK, "fold sync");
        ibtk_le_ctx_destroy(c2);
        for (int a = 0; a < 3; ++a) {
            auto hf = download(fs.ptr[a], asize("side", a, 1));
            save("f_phys_" + std::to_string(a) + ".bin", hf.data(), hf.size());
        }
        HC(hipFree(Sd));
    }
    std::printf("FACADE OK\n");
    return 0;
}
