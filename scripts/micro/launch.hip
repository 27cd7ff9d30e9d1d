// Back-to-back launch cost on MI355X: an (almost) empty kernel, n launches on one stream,
// for several grid / block / LDS shapes (the level-1 V-cycle launch is 512-8192 workgroups
// of 512 threads with 32 KB of LDS). Prints microseconds per launch.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k_empty(double *out, int flag) {
    extern __shared__ double lds[];
    if (flag) { lds[threadIdx.x] = 1.0; __syncthreads(); out[blockIdx.x] = lds[0]; }
}

__global__ void k_store(double *out, int n) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = 1.0;
}

int main() {
    double *buf = nullptr;
    hipMalloc(&buf, (size_t)64 << 20);
    hipStream_t s;
    hipStreamCreate(&s);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const int shapes[][3] = {{1, 64, 0}, {512, 512, 32768}, {1024, 512, 32768}, {8192, 512, 32768}, {8192, 256, 0}};
    for (auto &sh : shapes) {
        for (int warm = 0; warm < 10; ++warm) hipLaunchKernelGGL(k_empty, dim3(sh[0]), dim3(sh[1]), sh[2], s, buf, 0);
        hipEventRecord(a, s);
        const int n = 2000;
        for (int i = 0; i < n; ++i) hipLaunchKernelGGL(k_empty, dim3(sh[0]), dim3(sh[1]), sh[2], s, buf, 0);
        hipEventRecord(b, s);
        hipEventSynchronize(b);
        float ms = 0;
        hipEventElapsedTime(&ms, a, b);
        printf("empty grid=%d block=%d lds=%d: %.2f us per launch\n", sh[0], sh[1], sh[2], ms * 1e3 / n);
    }
    // a kernel that dirties 64 MB of L2 lines per launch
    const int n_el = 8 << 20, nb = n_el / 256;
    hipEventRecord(a, s);
    for (int i = 0; i < 500; ++i) hipLaunchKernelGGL(k_store, dim3(nb), dim3(256), 0, s, buf, n_el);
    hipEventRecord(b, s);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    printf("store 64 MB: %.2f us per launch (%.0f GB/s)\n", ms * 1e3 / 500, 64.0 * 1.048576e6 * 500 / (ms * 1e-3) / 1e9);
    return 0;
}
