// ubench_lds4.hip -- does a ds_add_f64 wave-instruction cost less when fewer lanes are
// active?  (Decides whether the spread's zero-weight adds -- a neighbour column's
// candidate adding its unowned stencil points with weight 0 -- are worth masking off.)
// Every pattern is conflict-free within each 16-lane group (lane 16 g + k hits bank
// class k); the patterns differ only in which lanes are active.  Standalone:
//   hipcc -O3 --offload-arch=gfx950 -o tools/ubench_lds4 tools/ubench_lds4.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#define CK(x)                                                                         \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

constexpr int NT = 512, ITERS = 4096, SLOTS = 2560, NPAT = 8;

// tab[wave][j][lane]: LDS slot of lane at step j (-1: lane inactive)
__global__ __launch_bounds__(NT) void k(const int* tab, double* out, unsigned long long* clk) {
    __shared__ double s[SLOTS];
    for (int i = threadIdx.x; i < SLOTS; i += NT) s[i] = 0.0;
    __syncthreads();
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const double v = 1.0 + lane * 1e-3;
    int a[NPAT];
    for (int j = 0; j < NPAT; ++j) a[j] = tab[(wave * NPAT + j) * 64 + lane];
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < ITERS; it += NPAT) {
#pragma unroll
        for (int j = 0; j < NPAT; ++j)
            if (a[j] >= 0) __hip_atomic_fetch_add(&s[a[j]], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        asm volatile("" ::: "memory");
    }
    __syncthreads();
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) clk[blockIdx.x] = t1 - t0;
    out[blockIdx.x * NT + threadIdx.x] = s[threadIdx.x];
}

int main() {
    int ncu = 0;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    std::mt19937 rng(7);
    struct Pat {
        const char* name;
        unsigned long long mask;  // active lanes
    };
    const Pat pats[] = {{"64 lanes (4 groups full)", ~0ull},
                        {"48 lanes (3 groups full)", 0x0000ffffffffffffull},
                        {"32 lanes (2 groups full)", 0x00000000ffffffffull},
                        {"16 lanes (1 group full)", 0x000000000000ffffull},
                        {"32 lanes (8 of 16 in each group)", 0x00ff00ff00ff00ffull},
                        {"16 lanes (4 of 16 in each group)", 0x000f000f000f000full},
                        {"48 lanes (12 of 16 in each group)", 0x0fff0fff0fff0fffull},
                        {"40 lanes (10 of 16 in each group)", 0x03ff03ff03ff03ffull}};
    const int NM = sizeof(pats) / sizeof(pats[0]);
    const int W = NT / 64;
    int* dtab;
    double* out;
    unsigned long long* clk;
    CK(hipMalloc(&dtab, sizeof(int) * W * NPAT * 64));
    const int nb = ncu;
    CK(hipMalloc(&out, sizeof(double) * nb * NT));
    CK(hipMalloc(&clk, sizeof(unsigned long long) * nb));
    std::vector<unsigned long long> h(nb);
    for (int mode = 0; mode < NM; ++mode) {
        std::vector<int> tab(W * NPAT * 64, -1);
        for (int w = 0; w < W; ++w)
            for (int j = 0; j < NPAT; ++j)
                for (int l = 0; l < 64; ++l) {
                    if (!((pats[mode].mask >> l) & 1ull)) continue;
                    const int row = rng() % 78;  // 78 rows of 32 doubles: 16-class pairs
                    tab[(w * NPAT + j) * 64 + l] = (row * 32 + (l & 15) + 16 * (rng() & 1)) % SLOTS;
                }
        CK(hipMemcpy(dtab, tab.data(), sizeof(int) * tab.size(), hipMemcpyHostToDevice));
        for (int rep = 0; rep < 2; ++rep) hipLaunchKernelGGL(k, dim3(nb), dim3(NT), 0, 0, dtab, out, clk);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(h.data(), clk, sizeof(unsigned long long) * nb, hipMemcpyDeviceToHost));
        double cyc = 0;
        for (int b = 0; b < nb; ++b) cyc += h[b];
        cyc /= nb;
        const double wi = (double)W * ITERS;
        printf("ds_add_f64 %-36s %.2f cyc/wave-instr/CU\n", pats[mode].name, cyc / wi);
    }
    return 0;
}
