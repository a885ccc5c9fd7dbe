// facade_test.cpp -- drives every overload form of the IBTK::LEInteractor C++ facade
// (include/ibtk_le/LEInteractor.h) on the GPU, the way LDataManager drives
// LEInteractor (LDataManager.cpp:625-660, 763-807), for Cell / Node / Side / Edge
// data on one periodic 3-D patch.  tests/test_gpu_boundary.py::test_cpp_facade
// writes the inputs (markers, fields, the index set's lists made by the oracle)
// into a directory, runs this program on it and compares what it writes back
// with the oracle.  Forms (LEInteractor.h:146-993):
//   a  LData views + index set      (interior list for interp, ghost list for spread)
//   b  raw device arrays + index set (same lists: must equal a bit for bit)
//   c  host std::vector, box filter  (markers whose cell is in the patch box, no shifts)
//   d  raw device arrays with sizes, box filter (must equal c bit for bit)
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
    // c: host vectors, the markers whose cell is in the patch box
    std::vector<double> Qh(init);
    LEInteractor::interpolate(Qh, Qdepth, hX, 3, u, patch, patch.box, "IB_4");
    save(std::string("Q_") + cname + "_c.bin", Qh.data(), nQ);
    zero_f();
    LEInteractor::spread(f, hQ2, Qdepth, hX, 3, patch, patch.box, "IB_4");
    LEInteractor::synchronize();
    save_f("c");
    // d: raw arrays with sizes
    HC(hipMemcpy(Qd, init.data(), sizeof(double) * nQ, hipMemcpyHostToDevice));
    LEInteractor::interpolate(Qd, (int)nQ, Qdepth, Xd, 3 * M, 3, u, patch, patch.box, "IB_4");
    LEInteractor::synchronize();
    h = download(Qd, nQ);
    save(std::string("Q_") + cname + "_d.bin", h.data(), nQ);
    zero_f();
    LEInteractor::spread(f, Sd, (int)nQ, Qdepth, Xd, 3 * M, 3, patch, patch.box, "IB_4");
    LEInteractor::synchronize();
    save_f("d");
    HC(hipFree(Qd));
    HC(hipFree(Sd));
}

int main(int argc, char** argv) {
    EXPECT(argc == 2, "usage: facade_test <dir>");
    D = argv[1];
    FILE* mf = std::fopen((D + "/meta.txt").c_str(), "r");
    EXPECT(mf && std::fscanf(mf, "%d %d %d %d %d %d", &N, &g, &M, &n_int, &n_all, &depth_c) == 6, "meta");
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
        Box other = patch.box.grow(1);
        LEInteractor::interpolate(Qv, Xv, idx, us, patch, other, pshift, "IB_4");
    } catch (const LEInteractorError& e) {
        thrown = e.code == IBTK_LE_ERR_ARG;
    }
    EXPECT(thrown, "index-set box other than the patch / ghost box throws");
    std::printf("FACADE OK\n");
    return 0;
}
