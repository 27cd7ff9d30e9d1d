// Microbenchmark: HBM rate of the level-1 launch's traffic mix without its arithmetic:
// read 2 planes-triples (tnew, RHS), write 3 (residual, tnew, tnew_nonlin), 16 B per lane,
// 1 pass over 8.4 M sub-elements (n_split = 5). Also 2R1W and 2R2W for reference.
#include <hip/hip_runtime.h>

#include <cstdio>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

template <int NW>
__global__ __launch_bounds__(256) void k_mix(const double *__restrict__ a, const double *__restrict__ b,
                                             double *__restrict__ o0, double *__restrict__ o1, double *__restrict__ o2,
                                             long pitch, long npairs) {
    const long p = (long)blockIdx.x * 256 + threadIdx.x;
    if (p >= npairs) return;
    const long s = 2 * p;
    double2 x[3], y[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        x[c] = *reinterpret_cast<const double2 *>(a + c * pitch + s);
        y[c] = *reinterpret_cast<const double2 *>(b + c * pitch + s);
    }
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        const double2 r = make_double2(x[c].x - y[c].x, x[c].y - y[c].y);
        const double2 q = make_double2(x[c].x + y[c].x, x[c].y + y[c].y);
        *reinterpret_cast<double2 *>(o0 + c * pitch + s) = r;
        if (NW >= 2) *reinterpret_cast<double2 *>(o1 + c * pitch + s) = q;
        if (NW >= 3) *reinterpret_cast<double2 *>(o2 + c * pitch + s) = make_double2(x[c].x * 2, y[c].y * 2);
    }
}

template <int NW>
int run(double *a, double *b, double *o0, double *o1, double *o2, long pitch, long npairs) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const unsigned g = (unsigned)((npairs + 255) / 256);
    for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(k_mix<NW>, dim3(g), dim3(256), 0, 0, a, b, o0, o1, o2, pitch, npairs);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < 20; ++i) hipLaunchKernelGGL(k_mix<NW>, dim3(g), dim3(256), 0, 0, a, b, o0, o1, o2, pitch, npairs);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = 1e3 * ms / 20, bytes = 2.0 * npairs * 24.0 * (2 + NW);
    printf("2R%dW: %8.1f us  %7.1f GB/s\n", NW, us, bytes / us * 1e-3);
    return 0;
}

int main() {
    const long N = 8192L << 10, pitch = N;
    double *a, *b, *o0, *o1, *o2;
    CK(hipMalloc(&a, 3 * pitch * 8));
    CK(hipMalloc(&b, 3 * pitch * 8));
    CK(hipMalloc(&o0, 3 * pitch * 8));
    CK(hipMalloc(&o1, 3 * pitch * 8));
    CK(hipMalloc(&o2, 3 * pitch * 8));
    CK(hipMemset(a, 0, 3 * pitch * 8));
    CK(hipMemset(b, 0, 3 * pitch * 8));
    int r = 0;
    for (int rep = 0; rep < 2; ++rep) {
        r |= run<1>(a, b, o0, o1, o2, pitch, N / 2);
        r |= run<2>(a, b, o0, o1, o2, pitch, N / 2);
        r |= run<3>(a, b, o0, o1, o2, pitch, N / 2);
    }
    return r;
}
