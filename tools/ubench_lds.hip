// ubench_lds.hip -- LDS f64 atomic / read throughput probes that decide the
// spread kernel's accumulation scheme.  Standalone:
//   hipcc -O3 --offload-arch=gfx950 -o tools/ubench_lds tools/ubench_lds.hip
// Prints cycles per wave-instruction per CU (clock from s_memtime vs s_memrealtime).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                     \
    do {                                                                          \
        hipError_t e_ = (x);                                                      \
        if (e_ != hipSuccess) {                                                   \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                              \
        }                                                                         \
    } while (0)

constexpr int NT = 256;
constexpr int ITERS = 2048;
constexpr int SLOTS = 2560;  // doubles in LDS (20 KB: 8 blocks per CU fit)

// mode 0: lane -> slot (lane + 64*wave)            conflict-free, distinct
// mode 1: 4x4x4 stencil in a 16-wide cube, row 16, plane 256 (unpadded)
// mode 2: 4x4x4 stencil, row 17, plane 17*17 (padded)
// mode 3: 4x4x4 stencil, row 20, plane 20*19+? (row 20, plane 400+4)
// mode 4: random slot per lane (hash), 4096 range
// mode 5: all lanes same slot
// mode 6: 4x4x4 stencil, row 16, plane 16*16+8 (pad planes only)
__device__ __forceinline__ int addr_of(int mode, int lane, int wave, int it) {
    const int i0 = lane & 3, i1 = (lane >> 2) & 3, i2 = lane >> 4;
    const int base = ((it * 37 + wave * 11) & 7);
    switch (mode) {
    case 0: return lane + 64 * wave;
    case 1: return base + i0 + 16 * i1 + 256 * i2 + 1024 * wave;
    case 2: return base + i0 + 17 * i1 + 289 * i2 + 1200 * wave;
    case 3: return base + i0 + 20 * i1 + 404 * i2 + 1400 * wave;
    case 4: {
        unsigned h = (unsigned)(lane * 2654435761u) ^ (unsigned)(it * 40503u) ^ (unsigned)(wave * 9973u);
        h ^= h >> 13;
        h *= 0x5bd1e995u;
        h ^= h >> 15;
        return (int)(h & 4095);
    }
    case 5: return 7;
    case 6: return base + i0 + 16 * i1 + 264 * i2 + 1100 * wave;
    default: return lane;
    }
}

template <int OP>
__global__ __launch_bounds__(NT) void k(int mode, double* out, unsigned long long* clk) {
    __shared__ double s[SLOTS];
    for (int i = threadIdx.x; i < SLOTS; i += NT) s[i] = 0.0;
    __syncthreads();
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const double v = 1.0 + lane * 1e-3;
    int a[8];
    for (int j = 0; j < 8; ++j) a[j] = addr_of(mode, lane, wave, j) % SLOTS;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    double acc = 0.0;
    for (int it = 0; it < ITERS; it += 8) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            if (OP == 0) {
                __hip_atomic_fetch_add(&s[a[j]], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            } else if (OP == 1) {
                acc += s[a[j] ^ (it & 1)];
            } else if (OP == 2) {
                float* sf = reinterpret_cast<float*>(s);
                __hip_atomic_fetch_add(&sf[a[j]], (float)v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
        }
        asm volatile("" ::: "memory");
    }
    __syncthreads();
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) {
        clk[2 * blockIdx.x] = t1 - t0;
        clk[2 * blockIdx.x + 1] = r1 - r0;
    }
    out[blockIdx.x * NT + threadIdx.x] = acc + s[threadIdx.x];
}

int main() {
    int ncu = 0;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    const char* names[] = {"lane->slot", "stencil row16", "stencil row17", "stencil row20", "random4096",
                           "same slot", "stencil row16 pl264"};
    const char* ops[] = {"ds_add_f64", "ds_read_b64", "ds_add_f32"};
    for (int bpc : {1, 2, 4, 8}) {
        const int nb = ncu * bpc;
        double* out;
        unsigned long long* clk;
        CK(hipMalloc(&out, sizeof(double) * nb * NT));
        CK(hipMalloc(&clk, sizeof(unsigned long long) * 2 * nb));
        unsigned long long* h = (unsigned long long*)malloc(sizeof(unsigned long long) * 2 * nb);
        for (int op = 0; op < 3; ++op) {
            for (int mode = 0; mode < 7; ++mode) {
                hipEvent_t e0, e1;
                CK(hipEventCreate(&e0));
                CK(hipEventCreate(&e1));
                for (int rep = 0; rep < 2; ++rep) {
                    CK(hipEventRecord(e0));
                    if (op == 0) hipLaunchKernelGGL(k<0>, dim3(nb), dim3(NT), 0, 0, mode, out, clk);
                    if (op == 1) hipLaunchKernelGGL(k<1>, dim3(nb), dim3(NT), 0, 0, mode, out, clk);
                    if (op == 2) hipLaunchKernelGGL(k<2>, dim3(nb), dim3(NT), 0, 0, mode, out, clk);
                    CK(hipEventRecord(e1));
                    CK(hipEventSynchronize(e1));
                }
                float ms = 0;
                CK(hipEventElapsedTime(&ms, e0, e1));
                CK(hipMemcpy(h, clk, sizeof(unsigned long long) * 2 * nb, hipMemcpyDeviceToHost));
                double cyc = 0, real = 0;
                for (int b = 0; b < nb; ++b) {
                    cyc += h[2 * b];
                    real += h[2 * b + 1];
                }
                cyc /= nb;
                real /= nb;
                const double ghz = cyc / real * 0.1;  // memrealtime = 100 MHz
                // wave-instructions per CU over the kernel = bpc * 4 waves * ITERS
                const double wi = (double)bpc * (NT / 64) * ITERS;
                const double cyc_per = cyc / wi;
                printf("blocks/CU %d  %-12s %-20s  %.2f cyc/wave-instr/CU (in-block), kernel %.3f ms, %.2f GHz\n", bpc,
                       ops[op], names[mode], cyc_per, ms, ghz);
                CK(hipEventDestroy(e0));
                CK(hipEventDestroy(e1));
            }
        }
        CK(hipFree(out));
        CK(hipFree(clk));
        free(h);
    }
    return 0;
}
