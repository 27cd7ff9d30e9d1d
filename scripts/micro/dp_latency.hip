// Microbenchmark: dependent-chain latency and issue rate of v_mul_f64 / v_add_f64
// on one wave (gfx950). Prints cycles per op for chains of ILP 1, 3, 6.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int ILP>
__global__ void chain(double *out, long long *cyc, double a, int n) {
    double x[ILP];
#pragma unroll
    for (int i = 0; i < ILP; ++i) x[i] = threadIdx.x + i;
    long long t0 = clock64();
    for (int k = 0; k < n; ++k) {
#pragma unroll
        for (int i = 0; i < ILP; ++i) x[i] = x[i] * a;
#pragma unroll
        for (int i = 0; i < ILP; ++i) x[i] = x[i] + a;
    }
    long long t1 = clock64();
    double s = 0;
#pragma unroll
    for (int i = 0; i < ILP; ++i) s += x[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int ILP>
void run(int waves_per_block, int blocks) {
    double *out;
    long long *cyc;
    hipMalloc(&out, sizeof(double) * 64 * waves_per_block * blocks);
    hipMalloc(&cyc, sizeof(long long) * blocks);
    const int n = 4096;
    hipLaunchKernelGGL(chain<ILP>, dim3(blocks), dim3(64 * waves_per_block), 0, 0, out, cyc, 1.0000001, n);
    hipLaunchKernelGGL(chain<ILP>, dim3(blocks), dim3(64 * waves_per_block), 0, 0, out, cyc, 1.0000001, n);
    hipDeviceSynchronize();
    long long c;
    hipMemcpy(&c, cyc, sizeof c, hipMemcpyDeviceToHost);
    printf("ILP %d waves/block %2d blocks %4d: %.2f cycles per dependent op-pair step, %.2f cycles per wave-instr\n",
           ILP, waves_per_block, blocks, (double)c / n / 2, (double)c / n / (2 * ILP));
    hipFree(out);
    hipFree(cyc);
}

int main() {
    run<1>(1, 1);
    run<3>(1, 1);
    run<6>(1, 1);
    run<3>(4, 1);
    run<3>(16, 1);
    run<6>(16, 1);
    run<3>(16, 256);
    return 0;
}
