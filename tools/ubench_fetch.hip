// ubench_fetch.hip -- calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE for the
// access widths the sweeps use (MI355X_MICROARCH.md, HBM section: the x2
// FETCH_SIZE correction is measured for 16-B-per-lane streaming reads only;
// "other access widths are uncalibrated").  Every kernel touches a known number
// of bytes of a 4 GiB buffer (far past the 256 MiB Infinity Cache), each byte
// once; the driver script divides the counters by these byte counts.
//
//   k_read8      8 B per lane, a wave reads 512 contiguous bytes
//   k_read16     16 B per lane (the guide's calibrated case)
//   k_rows8      8 B per lane over rows of 36 doubles (the interp ring's staged
//                plane rows: 288 B, starting at any 8-B offset), rows disjoint
//   k_write8     8 B per lane, contiguous
//   k_write16    16 B per lane, contiguous
//   k_write8_aos component c of 24-B records (Q(c, s) of AoS [M][3]): three
//                launches c = 0, 1, 2 each write a third of the records' bytes
// Prints one JSON object: kernel -> bytes touched per launch.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                       \
    do {                                                                            \
        hipError_t e = (x);                                                         \
        if (e != hipSuccess) {                                                      \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                  \
            exit(1);                                                                \
        }                                                                           \
    } while (0)

__global__ __launch_bounds__(256) void k_read8(const double* a, long n, double* out) {
    double s = 0.0;
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) s += a[i];
    if (s == 12345.678) out[blockIdx.x] = s;  // never true for the zero-filled input: keeps the loads
}
__global__ __launch_bounds__(256) void k_read16(const double2* a, long n2, double* out) {
    double s = 0.0;
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n2; i += (long)gridDim.x * 256) {
        const double2 v = a[i];
        s += v.x + v.y;
    }
    if (s == 12345.678) out[blockIdx.x] = s;
}
// rows of 36 doubles at a row stride of 1031 doubles (cfg4's side-array x extent):
// row r starts at r * 1031; lane l of the wave reads row element l, then l + 64
// (< 36 only for the first pass): 36 of 64 lanes busy, like the ring's plane loads
__global__ __launch_bounds__(256) void k_rows8(const double* a, long nrows, double* out) {
    const int lane = threadIdx.x & 63;
    const long wave = ((long)blockIdx.x * 256 + threadIdx.x) >> 6;
    const long nw = (long)gridDim.x * 4;
    double s = 0.0;
    for (long r = wave; r < nrows; r += nw)
        if (lane < 36) s += a[r * 1031 + lane];
    if (s == 12345.678) out[blockIdx.x] = s;
}
__global__ __launch_bounds__(256) void k_write8(double* a, long n) {
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) a[i] = 1.0;
}
__global__ __launch_bounds__(256) void k_write16(double2* a, long n2) {
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n2; i += (long)gridDim.x * 256) a[i] = make_double2(1.0, 2.0);
}
__global__ __launch_bounds__(256) void k_write8_aos(double* a, long nrec, int c) {
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < nrec; i += (long)gridDim.x * 256) a[3 * i + c] = 1.0;
}

int main() {
    const long bytes = 4L << 30;
    const long n = bytes / 8;
    double* a = nullptr;
    double* out = nullptr;
    CK(hipMalloc(&a, bytes));
    CK(hipMalloc(&out, 1 << 20));
    CK(hipMemset(a, 0, bytes));
    CK(hipDeviceSynchronize());
    const int grid = 256 * 16;
    const long nrows = n / 1031 - 1;
    for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL(k_read8, dim3(grid), dim3(256), 0, 0, a, n, out);
        hipLaunchKernelGGL(k_read16, dim3(grid), dim3(256), 0, 0, (const double2*)a, n / 2, out);
        hipLaunchKernelGGL(k_rows8, dim3(grid), dim3(256), 0, 0, a, nrows, out);
        hipLaunchKernelGGL(k_write8, dim3(grid), dim3(256), 0, 0, a, n);
        hipLaunchKernelGGL(k_write16, dim3(grid), dim3(256), 0, 0, (double2*)a, n / 2);
        for (int c = 0; c < 3; ++c) hipLaunchKernelGGL(k_write8_aos, dim3(grid), dim3(256), 0, 0, a, n / 3, c);
        CK(hipGetLastError());
        CK(hipDeviceSynchronize());
    }
    printf("{\"k_read8\": %ld, \"k_read16\": %ld, \"k_rows8\": %ld, \"k_write8\": %ld, \"k_write16\": %ld, "
           "\"k_write8_aos\": %ld}\n",
           bytes, bytes, nrows * 36 * 8, bytes, bytes, (n / 3) * 8);
    CK(hipFree(a));
    CK(hipFree(out));
    return 0;
}
