// ubench_lds2.hip -- ds_add_f64 cost versus the lane -> bank-class pattern,
// from host-generated address tables.  Decides how the spread sweep assigns
// candidates to lanes.  Standalone:
//   hipcc -O3 --offload-arch=gfx950 -o tools/ubench_lds2 tools/ubench_lds2.hip
// A double's bank pair is its index mod 32 ("class").
#include <hip/hip_runtime.h>

#include <algorithm>
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

constexpr int NT = 256, ITERS = 4096, SLOTS = 2560, NPAT = 8;

// tab[wave][j][lane]: LDS slot of lane at pattern j (-1: lane inactive)
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
    const char* names[] = {"distinct (L mod 32)",            // 0
                           "random",                         // 1
                           "q-distinct mod16, random rows",  // 2
                           "  + rotate class by j",          // 3
                           "  + x = c+j (no wrap, rows)",    // 4
                           "q-distinct, x in [0,31] mod16",  // 5
                           "q-distinct, trash rotate (row0)",// 6
                           "same addr every j per lane",     // 7
                           "q-distinct rows, +j, 44 busy"};  // 8
    const int NM = 9;
    int* dtab;
    double* out;
    unsigned long long* clk;
    CK(hipMalloc(&dtab, sizeof(int) * 4 * NPAT * 64));
    for (int bpc : {1, 2}) {
        const int nb = ncu * bpc;
        CK(hipMalloc(&out, sizeof(double) * nb * NT));
        CK(hipMalloc(&clk, sizeof(unsigned long long) * nb));
        std::vector<unsigned long long> h(nb);
        for (int mode = 0; mode < NM; ++mode) {
            std::vector<int> tab(4 * NPAT * 64, -1);
            for (int w = 0; w < 4; ++w) {
                // per-lane persistent choices (a "step"): class, row
                std::vector<int> cls(64), row(64), hi(64);
                for (int q = 0; q < 4; ++q) {
                    std::vector<int> perm(16);
                    for (int k = 0; k < 16; ++k) perm[k] = k;
                    std::shuffle(perm.begin(), perm.end(), rng);
                    for (int k = 0; k < 16; ++k) cls[16 * q + k] = perm[k];
                }
                for (int l = 0; l < 64; ++l) { row[l] = rng() % 60; hi[l] = rng() % 2; }
                for (int j = 0; j < NPAT; ++j) {
                    int* t = &tab[(w * NPAT + j) * 64];
                    for (int l = 0; l < 64; ++l) {
                        int ad = 0;
                        switch (mode) {
                        case 0: ad = l + 64 * w; break;
                        case 1: ad = rng() % 2048; break;
                        case 2: ad = row[l] * 32 + cls[l]; break;
                        case 3: ad = row[l] * 32 + ((cls[l] + j) & 15); break;
                        case 4: ad = row[l] * 32 + cls[l] + (j & 3); break;
                        case 5: ad = row[l] * 32 + cls[l] + 16 * hi[l]; break;
                        case 6: ad = 2000 + 16 * (l / 16) + ((cls[l] + j) & 15); break;
                        case 7: ad = 2000 + l; break;
                        case 8: ad = (l % 16) < 11 ? row[l] * 32 + cls[l] + (j & 3) : 2000 + 16 * (l / 16) + ((cls[l] + j) & 15); break;
                        }
                        t[l] = ad % SLOTS;
                    }
                }
            }
            CK(hipMemcpy(dtab, tab.data(), sizeof(int) * tab.size(), hipMemcpyHostToDevice));
            for (int rep = 0; rep < 2; ++rep) hipLaunchKernelGGL(k, dim3(nb), dim3(NT), 0, 0, dtab, out, clk);
            CK(hipDeviceSynchronize());
            CK(hipMemcpy(h.data(), clk, sizeof(unsigned long long) * nb, hipMemcpyDeviceToHost));
            double cyc = 0;
            for (int b = 0; b < nb; ++b) cyc += h[b];
            cyc /= nb;
            const double wi = (double)bpc * (NT / 64) * ITERS;
            printf("blocks/CU %d  ds_add_f64  %-26s %.2f cyc/wave-instr/CU\n", bpc, names[mode], cyc / wi);
        }
        CK(hipFree(out));
        CK(hipFree(clk));
    }
    return 0;
}
