// Microbenchmark: does the fp64 sweep arithmetic overlap the HBM stream?
// One streaming pass over x, b (3 fp64 planes each) -> out (3 planes), 72 B per
// sub-element, with K exact-order sweeps (pamg_device.h sweep) in between.
// Variants: one pair per thread (the per-step kernels' form) and a persistent
// form that prefetches the next pair before computing the current one.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#include "../../p-a_multigrids_amd/csrc/pamg_device.h"

using namespace pamg;
using namespace pamg::detail;

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

constexpr int LG = 10;   // 1024 sub-elements per un_ele (n_split = 5, level 1)

template <int K, int BS>
__global__ __launch_bounds__(BS) void k_plain(const double *__restrict__ x, const double *__restrict__ b,
                                              const double *__restrict__ stc, double *__restrict__ out,
                                              int64_t pitch, int64_t npairs, double rdt) {
    const int64_t p = (int64_t)blockIdx.x * BS + threadIdx.x;
    if (p >= npairs) return;
    const int64_t s = 2 * p;
    double2 xv[3], bv[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) { xv[c] = ld2(x + c * pitch + s); bv[c] = ld2(b + c * pitch + s); }
    Stc S;
    load_stc(stc + __builtin_amdgcn_readfirstlane((int)(s >> LG)) * kStcStride, S);
    double x0[3] = {xv[0].x, xv[1].x, xv[2].x}, x1[3] = {xv[0].y, xv[1].y, xv[2].y};
    const double b0[3] = {bv[0].x, bv[1].x, bv[2].x}, b1[3] = {bv[0].y, bv[1].y, bv[2].y};
    for (int k = 0; k < K; ++k) { sweep(S, rdt, b0, x0); sweep(S, rdt, b1, x1); }
#pragma unroll
    for (int c = 0; c < 3; ++c) st2(out + c * pitch + s, make_double2(x0[c], x1[c]));
}

// persistent: each thread walks pairs p, p + G, p + 2G, ...; the loads of the next
// pair are issued before the current pair's sweeps
template <int K, int BS>
__global__ __launch_bounds__(BS) void k_pref(const double *__restrict__ x, const double *__restrict__ b,
                                             const double *__restrict__ stc, double *__restrict__ out,
                                             int64_t pitch, int64_t npairs, double rdt) {
    const int64_t G = (int64_t)gridDim.x * BS;
    int64_t p = (int64_t)blockIdx.x * BS + threadIdx.x;
    if (p >= npairs) return;
    double2 xv[3], bv[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) { xv[c] = ld2(x + c * pitch + 2 * p); bv[c] = ld2(b + c * pitch + 2 * p); }
    for (; p < npairs; p += G) {
        const int64_t s = 2 * p;
        const int64_t q = p + G < npairs ? p + G : p;
        double2 xn[3], bn[3];
#pragma unroll
        for (int c = 0; c < 3; ++c) { xn[c] = ld2(x + c * pitch + 2 * q); bn[c] = ld2(b + c * pitch + 2 * q); }
        Stc S;
        load_stc(stc + __builtin_amdgcn_readfirstlane((int)(s >> LG)) * kStcStride, S);
        double x0[3] = {xv[0].x, xv[1].x, xv[2].x}, x1[3] = {xv[0].y, xv[1].y, xv[2].y};
        const double b0[3] = {bv[0].x, bv[1].x, bv[2].x}, b1[3] = {bv[0].y, bv[1].y, bv[2].y};
        for (int k = 0; k < K; ++k) { sweep(S, rdt, b0, x0); sweep(S, rdt, b1, x1); }
#pragma unroll
        for (int c = 0; c < 3; ++c) st2(out + c * pitch + s, make_double2(x0[c], x1[c]));
#pragma unroll
        for (int c = 0; c < 3; ++c) { xv[c] = xn[c]; bv[c] = bn[c]; }
    }
}

// compute only: K sweeps on register data, one store per thread
template <int K, int BS>
__global__ __launch_bounds__(BS) void k_compute(const double *__restrict__ stc, double *__restrict__ out, int64_t npairs,
                                                double rdt) {
    const int64_t p = (int64_t)blockIdx.x * BS + threadIdx.x;
    if (p >= npairs) return;
    Stc S;
    load_stc(stc + __builtin_amdgcn_readfirstlane((int)((2 * p) >> LG)) * kStcStride, S);
    double x0[3] = {1.0 * p, 2.0, 3.0}, x1[3] = {4.0, 5.0 * p, 6.0};
    const double b0[3] = {1, 2, 3}, b1[3] = {3, 2, 1};
    for (int k = 0; k < K; ++k) { sweep(S, rdt, b0, x0); sweep(S, rdt, b1, x1); }
    out[p] = x0[0] + x0[1] + x0[2] + x1[0] + x1[1] + x1[2];
}

template <int K, int BS>
int run(const char *tag, int variant, const double *x, const double *b, const double *stc, double *out, int64_t pitch,
        int64_t npairs, int cus) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const unsigned gplain = (unsigned)((npairs + BS - 1) / BS);
    const unsigned gpers = (unsigned)cus * (2048 / BS);
    auto launch = [&]() {
        if (variant == 0) hipLaunchKernelGGL((k_plain<K, BS>), dim3(gplain), dim3(BS), 0, 0, x, b, stc, out, pitch, npairs, 8e4);
        else if (variant == 1) hipLaunchKernelGGL((k_pref<K, BS>), dim3(gpers), dim3(BS), 0, 0, x, b, stc, out, pitch, npairs, 8e4);
        else hipLaunchKernelGGL((k_compute<K, BS>), dim3(gplain), dim3(BS), 0, 0, stc, out, npairs, 8e4);
    };
    for (int i = 0; i < 3; ++i) launch();
    CK(hipDeviceSynchronize());
    const int reps = 20;
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < reps; ++i) launch();
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = 1e3 * ms / reps;
    const double bytes = 72.0 * 2 * npairs;
    printf("%-8s K=%2d BS=%4d  %8.1f us  %7.1f GB/s (72 B/sub-element)\n", tag, K, BS, us, variant == 2 ? 0.0 : bytes / us * 1e-3);
    return 0;
}

template <int BS>
int sweepK(int variant, const char *tag, const double *x, const double *b, const double *stc, double *out,
           int64_t pitch, int64_t npairs, int cus) {
    int r = 0;
    r |= run<0, BS>(tag, variant, x, b, stc, out, pitch, npairs, cus);
    r |= run<1, BS>(tag, variant, x, b, stc, out, pitch, npairs, cus);
    r |= run<2, BS>(tag, variant, x, b, stc, out, pitch, npairs, cus);
    r |= run<4, BS>(tag, variant, x, b, stc, out, pitch, npairs, cus);
    r |= run<8, BS>(tag, variant, x, b, stc, out, pitch, npairs, cus);
    r |= run<16, BS>(tag, variant, x, b, stc, out, pitch, npairs, cus);
    return r;
}

int main() {
    const int64_t U = 8192, N = U << LG, pitch = N;
    double *x, *b, *out, *stc;
    CK(hipMalloc(&x, 3 * pitch * 8));
    CK(hipMalloc(&b, 3 * pitch * 8));
    CK(hipMalloc(&out, 3 * pitch * 8));
    CK(hipMalloc(&stc, U * kStcStride * 8));
    std::vector<double> h(3 * pitch);
    for (int64_t i = 0; i < 3 * pitch; ++i) h[i] = 1e-3 * (double)((i * 2654435761u) % 1000);
    CK(hipMemcpy(x, h.data(), 3 * pitch * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(b, h.data(), 3 * pitch * 8, hipMemcpyHostToDevice));
    std::vector<double> hs(U * kStcStride);
    for (int64_t u = 0; u < U; ++u)
        for (int q = 0; q < kStcStride; ++q) hs[u * kStcStride + q] = (q < 18) ? 1e-6 * (1 + (q % 3 == q / 3 % 3)) : 0.1;
    CK(hipMemcpy(stc, hs.data(), hs.size() * 8, hipMemcpyHostToDevice));
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    printf("CUs %d, N %lld sub-elements\n", cus, (long long)N);
    int r = 0;
    r |= sweepK<256>(2, "compute", x, b, stc, out, pitch, N / 2, cus);
    r |= sweepK<256>(0, "plain", x, b, stc, out, pitch, N / 2, cus);
    r |= sweepK<512>(0, "plain", x, b, stc, out, pitch, N / 2, cus);
    r |= sweepK<256>(1, "prefetch", x, b, stc, out, pitch, N / 2, cus);
    r |= sweepK<512>(1, "prefetch", x, b, stc, out, pitch, N / 2, cus);
    return r;
}
