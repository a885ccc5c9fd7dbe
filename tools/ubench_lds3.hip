// ubench_lds3.hip -- ds_add_f64 cost of the spread's per-chunk add patterns:
// 64 lanes with random stencil starts (x in [-3, 31], y in [-3, 15]), 4x4 rows
// of 4 adds (one plane), under the lane dealings the spread sweep can use.
//   hipcc -O3 --offload-arch=gfx950 -o tools/ubench_lds3 tools/ubench_lds3.hip
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

constexpr int NT = 64, NI = 64, NTAB = 8, SLOTS = 4096, REP = 64;

// tab[t][i][lane]: LDS slot (-1 inactive) of lane at instruction i of table t
__global__ __launch_bounds__(NT) void k(const int* tab, double* out, unsigned long long* clk) {
    __shared__ double s[SLOTS];
    for (int i = threadIdx.x; i < SLOTS; i += NT) s[i] = 0.0;
    __syncthreads();
    const int lane = threadIdx.x;
    const double v = 1.0 + lane * 1e-3;
    const int* tb = tab + (blockIdx.x % NTAB) * NI * 64;
    int a[NI];
    for (int i = 0; i < NI; ++i) a[i] = tb[i * 64 + lane];
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < REP; ++it) {
#pragma unroll
        for (int i = 0; i < NI; ++i)
            if (a[i] >= 0) __hip_atomic_fetch_add(&s[a[i]], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
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
    std::mt19937 rng(11);
    const char* names[] = {"random lanes, RS 32", "dealt x mod 16 (RR), RS 32", "blk4 x mod 4 + rot, RS 36",
                           "blk4 x mod 4 + rot, RS 40", "no conflict (lane-distinct mod 32)", "dealt x mod 32 (RR 2x32), RS 32"};
    const int NM = 6;
    int* dtab;
    double* out;
    unsigned long long* clk;
    CK(hipMalloc(&dtab, sizeof(int) * NTAB * NI * 64));
    for (int wpc : {1, 4, 7}) {
        const int nb = ncu * wpc;
        CK(hipMalloc(&out, sizeof(double) * nb * NT));
        CK(hipMalloc(&clk, sizeof(unsigned long long) * nb));
        std::vector<unsigned long long> h(nb);
        for (int mode = 0; mode < NM; ++mode) {
            std::vector<int> tab(NTAB * NI * 64, -1);
            for (int t = 0; t < NTAB; ++t) {
                std::vector<int> x(64), y(64), ord(64), q(64, 0);
                for (int l = 0; l < 64; ++l) { x[l] = (int)(rng() % 35) - 3; y[l] = (int)(rng() % 19) - 3; }
                for (int l = 0; l < 64; ++l) ord[l] = l;
                int RS = mode == 2 ? 36 : (mode == 3 ? 40 : 32);
                auto cls16 = [&](int l) { return ((x[l] % 16) + 16) % 16; };
                auto cls32 = [&](int l) { return ((x[l] % 32) + 32) % 32; };
                auto res4 = [&](int l) { return ((x[l] % 4) + 4) % 4; };
                std::vector<int> lane_of(64);  // dealt position -> source
                if (mode == 0 || mode == 4) {
                    for (int l = 0; l < 64; ++l) lane_of[l] = l;
                } else if (mode == 1 || mode == 5) {
                    std::stable_sort(ord.begin(), ord.end(), [&](int a, int b) { return mode == 1 ? cls16(a) < cls16(b) : cls32(a) < cls32(b); });
                    for (int k = 0; k < 64; ++k) {
                        int tl = mode == 1 ? (k % 4) * 16 + k / 4 : (k % 2) * 32 + k / 2;
                        lane_of[tl] = ord[k];
                    }
                } else {
                    std::stable_sort(ord.begin(), ord.end(), [&](int a, int b) { return res4(a) < res4(b); });
                    for (int k = 0; k < 64; ++k) lane_of[((k >> 2) & 3) * 16 + (k >> 4) * 4 + (k & 3)] = ord[k];
                    for (int L = 0; L < 64; ++L) {  // q = rank among same residue in group
                        int c = 0;
                        for (int M = L & 48; M < L; ++M) c += res4(lane_of[M]) == res4(lane_of[L]);
                        q[L] = c & 3;
                    }
                }
                for (int L = 0; L < 64; ++L) {
                    const int l = lane_of[L];
                    const int ox = x[l], oy = y[l];
                    const int fl = (int)std::floor(ox / 4.0);
                    const int rot = mode >= 2 && mode <= 3 ? (((q[L] - oy - fl) % 4) + 4) % 4 : 0;
                    for (int j = 0; j < 4; ++j)
                        for (int i1 = 0; i1 < 4; ++i1)  // i2 plane fixed: 16 rows x 4 adds = 64 instr
                            for (int i0 = 0; i0 < 4; ++i0) {
                                const int ins = (j * 4 + i1) * 4 + i0;
                                const int r = (i1 + rot) & 3;
                                int ad = 64 + 600 * j + RS * (oy + 3 + r) + ox + 3 + i0;
                                if (mode == 4) ad = 64 + L + 64 * ((ins + L) & 7);
                                tab[(t * NI + ins) * 64 + L] = ad % SLOTS;
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
            printf("waves/CU %d  %-36s %.2f cyc/instr/CU\n", wpc, names[mode], cyc / (double)(REP * NI) / wpc);
        }
        CK(hipFree(out));
        CK(hipFree(clk));
    }
    return 0;
}
