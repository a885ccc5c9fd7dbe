// facade_test.cpp -- exercises the IBTK::LEInteractor C++ facade on the GPU the way
// LDataManager drives LEInteractor (LDataManager.cpp:625-660, 763-807): side-centred
// data on one periodic patch, interior index list for interpolation, ghost-box
// list (with periodic images) for spreading.  Prints "FACADE OK" on success.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
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

int main() {
    const int N = 16, g = 3, M = 500;
    PatchView patch;
    patch.box.ndim = 3;
    for (int d = 0; d < 3; ++d) {
        patch.box.lower[d] = 0;
        patch.box.upper[d] = N - 1;
        patch.dx[d] = 1.0 / N;
        patch.x_lower[d] = 0.0;
        patch.x_upper[d] = 1.0;
    }
    SideDataView u, f;
    u.box = f.box = patch.box;
    size_t sz[3];
    for (int a = 0; a < 3; ++a) {
        sz[a] = 1;
        for (int d = 0; d < 3; ++d) sz[a] *= (size_t)(N + 2 * g + (d == a));
        HC(hipMalloc(&u.ptr[a], sz[a] * 8));
        HC(hipMalloc(&f.ptr[a], sz[a] * 8));
        std::vector<double> h(sz[a], 2.0 + a);
        HC(hipMemcpy(u.ptr[a], h.data(), sz[a] * 8, hipMemcpyHostToDevice));
        HC(hipMemset(f.ptr[a], 0, sz[a] * 8));
    }
    for (int d = 0; d < 3; ++d) u.ghost[d] = f.ghost[d] = g;
    std::mt19937_64 rng(3);
    std::uniform_real_distribution<double> U01(0.0, 1.0);
    std::vector<double> hX(3 * M), hF(3 * M);
    for (auto& v : hX) v = U01(rng);
    for (auto& v : hF) v = U01(rng) - 0.5;
    double *X, *Q, *Fd;
    HC(hipMalloc(&X, 24 * M));
    HC(hipMalloc(&Q, 24 * M));
    HC(hipMalloc(&Fd, 24 * M));
    HC(hipMemcpy(X, hX.data(), 24 * M, hipMemcpyHostToDevice));
    HC(hipMemcpy(Fd, hF.data(), 24 * M, hipMemcpyHostToDevice));

    // index set: interior = identity, ghost box = identity + periodic images
    ibtk_le_ctx ctx;
    EXPECT(ibtk_le_ctx_create(0, nullptr, &ctx) == 0, "ctx");
    ibtk_le_patch_geom geom{};
    geom.ndim = 3;
    for (int d = 0; d < 3; ++d) {
        geom.iupper[d] = N - 1;
        geom.gcw[d] = g;
        geom.dx[d] = 1.0 / N;
        geom.x_upper[d] = 1.0;
    }
    int *idx_int, *idx_all;
    double *xs_int, *xs_all;
    HC(hipMalloc(&idx_int, 4 * M));
    HC(hipMalloc(&xs_int, 24 * M));
    HC(hipMalloc(&idx_all, 4 * 27 * M));
    HC(hipMalloc(&xs_all, 24 * 27 * M));
    int n_int = 0, n_all = 0;
    EXPECT(ibtk_le_periodic_index_list(ctx, &geom, X, M, 0, nullptr, idx_int, xs_int, M, &n_int) == 0, "interior list");
    EXPECT(ibtk_le_periodic_index_list(ctx, &geom, X, M, g, nullptr, idx_all, xs_all, 27 * M, &n_all) == 0, "ghost list");
    EXPECT(n_int == M && n_all > M, "list sizes");
    LIndexSetView idx;
    idx.ghost_box = patch.box.grow(g);
    idx.local_indices = idx_all;
    idx.periodic_shifts = xs_all;
    idx.n = n_all;
    idx.interior_local_indices = idx_int;
    idx.interior_periodic_shifts = xs_int;
    idx.n_interior = n_int;
    const int pshift[3] = {N, N, N};

    EXPECT(LEInteractor::getStencilSize("IB_4") == 4 && LEInteractor::getMinimumGhostWidth("IB_6") == 4, "stencil");
    LDataView Qv{Q, 3, M}, Xv{X, 3, M}, Fv{Fd, 3, M};
    LEInteractor::interpolate(Qv, Xv, idx, u, patch, patch.box, pshift, "IB_4");
    LEInteractor::spread(f, Fv, Xv, idx, patch, idx.ghost_box, pshift, "IB_4");
    LEInteractor::synchronize();
    std::vector<double> hQ(3 * M);
    HC(hipMemcpy(hQ.data(), Q, 24 * M, hipMemcpyDeviceToHost));
    for (int s = 0; s < M; ++s)
        for (int a = 0; a < 3; ++a) EXPECT(std::fabs(hQ[3 * s + a] - (2.0 + a)) < 1e-13, "interp of a constant");
    // spreading with periodic images: the interior sum times h^3 equals sum F
    for (int a = 0; a < 3; ++a) {
        std::vector<double> h(sz[a]);
        HC(hipMemcpy(h.data(), f.ptr[a], sz[a] * 8, hipMemcpyDeviceToHost));
        const int n0 = N + 2 * g + (a == 0), n1 = N + 2 * g + (a == 1);
        double tot = 0.0, ref = 0.0;
        for (int k = g; k < g + N; ++k)
            for (int j = g; j < g + N; ++j)
                for (int i = g; i < g + N; ++i) tot += h[(size_t)(k * n1 + j) * n0 + i];
        for (int s = 0; s < M; ++s) ref += hF[3 * s + a];
        EXPECT(std::fabs(tot / (N * N * N) - ref) < 1e-11, "spread conserves the total");
    }
    // X-only overload over the patch box gives the same interpolant
    HC(hipMemset(Q, 0, 24 * M));
    LEInteractor::interpolate(Q, 3, X, 3, 3 * M, u, patch, patch.box, "IB_4");
    LEInteractor::synchronize();
    HC(hipMemcpy(hQ.data(), Q, 24 * M, hipMemcpyDeviceToHost));
    for (int s = 0; s < M; ++s) EXPECT(std::fabs(hQ[3 * s] - 2.0) < 1e-13, "X-only interp");
    // error conventions
    bool thrown = false;
    try {
        LEInteractor::interpolate(Qv, Xv, idx, u, patch, patch.box, pshift, "NOT_A_KERNEL");
    } catch (const LEInteractorError& e) {
        thrown = e.code == IBTK_LE_ERR_UNKNOWN_KERNEL;
    }
    EXPECT(thrown, "unknown kernel throws");
    thrown = false;
    try {
        LEInteractor::interpolate(Qv, Xv, idx, u, patch, patch.box, pshift, "IB_6");  // needs 4 ghosts
    } catch (const LEInteractorError& e) {
        thrown = e.code == IBTK_LE_ERR_GHOST_WIDTH;
    }
    EXPECT(thrown, "ghost width throws");
    thrown = false;
    try {
        LDataView Q2{Q, 2, M};
        LEInteractor::interpolate(Q2, Xv, idx, u, patch, patch.box, pshift, "IB_4");
    } catch (const LEInteractorError& e) {
        thrown = e.code == IBTK_LE_ERR_DEPTH;
    }
    EXPECT(thrown, "depth mismatch throws");
    std::printf("FACADE OK\n");
    return 0;
}
