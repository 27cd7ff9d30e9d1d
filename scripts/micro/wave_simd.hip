// Probe: which SIMD each wave of a 512-thread workgroup lands on (HW_REG_HW_ID), for a grid
// of 8192 workgroups as the resident V-cycle launch uses. Prints, per wave index of the
// workgroup, the histogram of its SIMD id relative to wave 0's, and the histogram of wave 0's
// SIMD id. Build: hipcc --offload-arch=gfx950 -O2 wave_simd.hip -o /tmp/wave_simd
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ __launch_bounds__(512) void probe(unsigned *hw, double *sink, int n) {
    unsigned id;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(id));
    double x = threadIdx.x;
    for (int i = 0; i < n; ++i) x = __builtin_fma(x, 1.0000001, 0.5);   // keep the waves resident a while
    if ((threadIdx.x & 63) == 0) hw[blockIdx.x * 8 + (threadIdx.x >> 6)] = id;   // vector store
    if (x == 12345.0) sink[threadIdx.x] = x;
}

int main() {
    const int grid = 8192;
    unsigned *d;
    double *sink;
    hipMalloc(&d, grid * 8 * sizeof(unsigned));
    hipMalloc(&sink, 512 * sizeof(double));
    hipLaunchKernelGGL(probe, dim3(grid), dim3(512), 0, 0, d, sink, 20000);
    hipDeviceSynchronize();
    std::vector<unsigned> h(grid * 8);
    hipMemcpy(h.data(), d, h.size() * sizeof(unsigned), hipMemcpyDeviceToHost);
    int rel[8][4] = {}, w0[4] = {};
    for (int b = 0; b < grid; ++b) {
        const int s0 = (h[b * 8] >> 4) & 3;
        w0[s0]++;
        for (int w = 0; w < 8; ++w) rel[w][(((h[b * 8 + w] >> 4) & 3) - s0 + 4) & 3]++;
    }
    printf("wave 0 SIMD histogram: %d %d %d %d\n", w0[0], w0[1], w0[2], w0[3]);
    for (int w = 0; w < 8; ++w) printf("wave %d SIMD - wave0 SIMD: %5d %5d %5d %5d\n", w, rel[w][0], rel[w][1], rel[w][2], rel[w][3]);
    printf("first 8 workgroups (hw_id of waves 0..7):\n");
    for (int b = 0; b < 8; ++b) {
        for (int w = 0; w < 8; ++w) printf(" %08x", h[b * 8 + w]);
        printf("\n");
    }
    return 0;
}
