// ubench_glds.hip -- checks the LDS-DMA primitive the sweep kernels use
// (__builtin_amdgcn_global_load_lds, size 4, per-lane source addresses,
// misaligned rows) and a counted manual vmcnt wait.  Standalone:
//   hipcc -O3 --offload-arch=gfx950 -o tools/ubench_glds tools/ubench_glds.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                 \
    do {                                                                                      \
        hipError_t e_ = (x);                                                                  \
        if (e_ != hipSuccess) {                                                               \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));         \
            exit(1);                                                                          \
        }                                                                                     \
    } while (0)

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void gbl_void_t;

__device__ __forceinline__ void glds4(const void* g, void* l) {
    __builtin_amdgcn_global_load_lds((gbl_void_t*)g, (lds_void_t*)l, 4, 0, 0);
}

// each wave: DMA 16 rows of 32 doubles (row r of the source starts at r*stride+off,
// odd stride => misaligned rows), XOR-swizzled through the source address, then
// read back un-swizzled and written out.
__global__ __launch_bounds__(64) void k_copy(const double* src, int stride, int off, double* dst) {
    __shared__ double ring[512];
    const int lane = threadIdx.x;
    const double* base = src + (size_t)blockIdx.x * 16 * stride + off;
    for (int y = 0; y < 16; ++y) {
        const int p = lane >> 1, half = lane & 1;
        const int x = p ^ ((y & 3) << 2);
        const char* g = (const char*)(base + (size_t)y * stride + x) + 4 * half;
        glds4(g, (char*)ring + 256 * y);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    for (int k = 0; k < 8; ++k) {
        const int q = lane + 64 * k, x = q & 31, y = q >> 5;
        dst[(size_t)blockIdx.x * 512 + q] = ring[y * 32 + (x ^ ((y & 3) << 2))];
    }
}

int main() {
    const int nb = 4096, stride = 1031, off = 3;
    const size_t n = (size_t)nb * 16 * stride + 64;
    std::vector<double> h(n);
    for (size_t i = 0; i < n; ++i) h[i] = (double)i * 0.5 + 1.0;
    double *s, *d;
    CK(hipMalloc(&s, n * 8));
    CK(hipMalloc(&d, (size_t)nb * 512 * 8));
    CK(hipMemcpy(s, h.data(), n * 8, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_copy, dim3(nb), dim3(64), 0, 0, s, stride, off, d);
    CK(hipDeviceSynchronize());
    std::vector<double> o((size_t)nb * 512);
    CK(hipMemcpy(o.data(), d, o.size() * 8, hipMemcpyDeviceToHost));
    long bad = 0;
    for (int b = 0; b < nb; ++b)
        for (int q = 0; q < 512; ++q) {
            const int x = q & 31, y = q >> 5;
            const double want = h[(size_t)b * 16 * stride + off + (size_t)y * stride + x];
            if (o[(size_t)b * 512 + q] != want) ++bad;
        }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0));
    for (int r = 0; r < 20; ++r) hipLaunchKernelGGL(k_copy, dim3(nb), dim3(64), 0, 0, s, stride, off, d);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("glds copy: mismatches %ld of %d, %.3f ms/launch\n", bad, nb * 512, ms / 20);
    return bad ? 1 : 0;
}
