// Microbenchmark: the coarsest level's smoother chain (k_vc_resb wave 4) in three forms, on
// one workgroup (an idle chip: the irregular.msh n_split = 6 case, 44 tiles on 256 CUs).
//   rows   one lane per sub-element, the contracted sweep (12 fma, depth 4, ILP 3): the kernel's form
//   quad   a sub-element's three rows on three lanes of a quad (3 + 1 fma per lane, depth 4), the new
//          iterate broadcast inside the quad with DPP quad_perm after every sweep
//   affine x' = B x + c (9 fma, depth 3): a different rounding, for scale only
// Prints cycles (clock64) per sweep. Build: hipcc --offload-arch=gfx950 -O3 chain_split.hip
#include <hip/hip_runtime.h>
#include <cstdio>

__device__ __forceinline__ double bcast(double v, int q) {
    const int lo = __double2loint(v), hi = __double2hiint(v);
    int rl, rh;
    if (q == 0) {
        rl = __builtin_amdgcn_update_dpp(0, lo, 0x00, 0xF, 0xF, false);
        rh = __builtin_amdgcn_update_dpp(0, hi, 0x00, 0xF, 0xF, false);
    } else if (q == 1) {
        rl = __builtin_amdgcn_update_dpp(0, lo, 0x55, 0xF, 0xF, false);
        rh = __builtin_amdgcn_update_dpp(0, hi, 0x55, 0xF, 0xF, false);
    } else {
        rl = __builtin_amdgcn_update_dpp(0, lo, 0xAA, 0xF, 0xF, false);
        rh = __builtin_amdgcn_update_dpp(0, hi, 0xAA, 0xF, 0xF, false);
    }
    return __hiloint2double(rh, rl);
}

__global__ void k_rows(const double *A, double *out, long long *cyc, int n) {
    double a[9], w[3], x[3], b[3];
    for (int q = 0; q < 9; ++q) a[q] = A[q];
    for (int q = 0; q < 3; ++q) { w[q] = A[9 + q]; x[q] = threadIdx.x + q; b[q] = 0.5 * q; }
    const long long t0 = clock64();
    for (int k = 0; k < n; ++k) {
        double t[3];
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            t[i] = __builtin_fma(-a[3 * i], x[0], b[i]);
            t[i] = __builtin_fma(-a[3 * i + 1], x[1], t[i]);
            t[i] = __builtin_fma(-a[3 * i + 2], x[2], t[i]);
        }
#pragma unroll
        for (int i = 0; i < 3; ++i) x[i] = __builtin_fma(w[i], t[i], x[i]);
    }
    const long long t1 = clock64();
    out[threadIdx.x] = x[0] + x[1] + x[2];
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

__global__ void k_quad(const double *A, double *out, long long *cyc, int n) {
    const int r = threadIdx.x & 3, rr = r < 3 ? r : 2;   // lane 3 of a quad repeats row 2
    const double a0 = A[3 * rr], a1 = A[3 * rr + 1], a2 = A[3 * rr + 2], w = A[9 + rr];
    const double b = 0.5 * rr;
    double x0 = (threadIdx.x >> 2), x1 = x0 + 1, x2 = x0 + 2;
    double xr = rr == 0 ? x0 : rr == 1 ? x1 : x2;
    const long long t0 = clock64();
    for (int k = 0; k < n; ++k) {
        double t = __builtin_fma(-a0, x0, b);
        t = __builtin_fma(-a1, x1, t);
        t = __builtin_fma(-a2, x2, t);
        xr = __builtin_fma(w, t, xr);
        x0 = bcast(xr, 0);
        x1 = bcast(xr, 1);
        x2 = bcast(xr, 2);
    }
    const long long t1 = clock64();
    out[threadIdx.x] = xr;
    if (threadIdx.x == 0) cyc[1] = t1 - t0;
}

__global__ void k_affine(const double *A, double *out, long long *cyc, int n) {
    double m[9], x[3], c[3];
    for (int q = 0; q < 9; ++q) m[q] = A[q];
    for (int q = 0; q < 3; ++q) { x[q] = threadIdx.x + q; c[q] = 0.5 * q; }
    const long long t0 = clock64();
    for (int k = 0; k < n; ++k) {
        double y[3];
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            y[i] = __builtin_fma(m[3 * i], x[0], c[i]);
            y[i] = __builtin_fma(m[3 * i + 1], x[1], y[i]);
            y[i] = __builtin_fma(m[3 * i + 2], x[2], y[i]);
        }
#pragma unroll
        for (int i = 0; i < 3; ++i) x[i] = y[i];
    }
    const long long t1 = clock64();
    out[threadIdx.x] = x[0] + x[1] + x[2];
    if (threadIdx.x == 0) cyc[2] = t1 - t0;
}

int main() {
    const double hA[12] = {0.31, -0.02, 0.01, -0.03, 0.29, 0.02, 0.01, -0.01, 0.33, 0.9, 0.8, 0.85};
    double *A, *out;
    long long *cyc, h[3];
    hipMalloc(&A, sizeof hA);
    hipMalloc(&out, 256 * sizeof(double));
    hipMalloc(&cyc, 3 * sizeof(long long));
    hipMemcpy(A, hA, sizeof hA, hipMemcpyHostToDevice);
    const int n = 4096;
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(k_rows, dim3(1), dim3(64), 0, 0, A, out, cyc, n);
        hipLaunchKernelGGL(k_quad, dim3(1), dim3(256), 0, 0, A, out, cyc, n);
        hipLaunchKernelGGL(k_affine, dim3(1), dim3(64), 0, 0, A, out, cyc, n);
    }
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    hipMemcpy(h, cyc, sizeof h, hipMemcpyDeviceToHost);
    printf("rows   (1 lane / sub-element, 12 fma depth 4): %.1f cycles per sweep\n", (double)h[0] / n);
    printf("quad   (3 rows on a quad + DPP broadcast)    : %.1f cycles per sweep\n", (double)h[1] / n);
    printf("affine (9 fma depth 3, other rounding)       : %.1f cycles per sweep\n", (double)h[2] / n);
    return 0;
}
