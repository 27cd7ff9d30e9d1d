// Probe: can a stream wait (hipStreamWaitValue64) on a counter that a running kernel on another
// stream raises with a system-scope atomic? (the resident call's per-cycle exchange, pamg_api.cpp
// vcycle_fused, halo_exchange = 1). Signal memory (hipMallocSignalMemory) and, for comparison,
// plain device memory. Every wait is bounded on the host (hipStreamQuery polling, 5 s).
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <thread>

__global__ void k_raise(unsigned long long *sig, int rounds, long long spin) {
    for (int r = 0; r < rounds; ++r) {
        const long long t0 = wall_clock64();
        while (wall_clock64() - t0 < spin) {
        }
        __syncthreads();
        if (threadIdx.x == 0) __hip_atomic_fetch_add(sig, 1ull, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

__global__ void k_mark(unsigned *out, int i, long long *when) {
    if (threadIdx.x == 0) {
        out[i] = 1;
        when[i] = wall_clock64();
    }
}

static bool wait_stream(hipStream_t s, double sec) {
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
        const hipError_t e = hipStreamQuery(s);
        if (e == hipSuccess) return true;
        if (e != hipErrorNotReady) {
            printf("stream error %s\n", hipGetErrorString(e));
            return false;
        }
        if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > sec) return false;
        std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
}

static int probe(const char *name, unsigned long long *sig) {
    hipStream_t a, b;
    (void)hipStreamCreateWithFlags(&a, hipStreamNonBlocking);
    (void)hipStreamCreateWithFlags(&b, hipStreamNonBlocking);
    unsigned long long base = 0;
    (void)hipMemcpy(&base, sig, sizeof base, hipMemcpyDeviceToHost);
    unsigned *out;
    long long *when;
    (void)hipMalloc(&out, 64 * sizeof(unsigned));
    (void)hipMalloc(&when, 64 * sizeof(long long));
    (void)hipMemset(out, 0, 64 * sizeof(unsigned));
    const int rounds = 8;
    const long long spin = 100000;   // wall_clock64 ticks (100 MHz: 1 ms)
    hipLaunchKernelGGL(k_raise, dim3(64), dim3(256), 0, a, sig, rounds, spin);
    hipError_t e = hipSuccess;
    for (int r = 0; r < rounds; ++r) {
        // every workgroup raises the counter once per round: round r is complete at base + 64 (r + 1)
        e = hipStreamWaitValue64(b, sig, base + 64ull * (r + 1), hipStreamWaitValueGte, ~0ull);
        if (e != hipSuccess) break;
        hipLaunchKernelGGL(k_mark, dim3(1), dim3(64), 0, b, out, r, when);
    }
    printf("%s: base %llu, wait enqueue %s\n", name, base, hipGetErrorString(e));
    const bool ok_b = e == hipSuccess && wait_stream(b, 5.0);
    const bool ok_a = wait_stream(a, 5.0);
    unsigned h[64] = {};
    long long w[64] = {};
    (void)hipMemcpy(h, out, sizeof h, hipMemcpyDeviceToHost);
    (void)hipMemcpy(w, when, sizeof w, hipMemcpyDeviceToHost);
    unsigned long long fin = 0;
    (void)hipMemcpy(&fin, sig, sizeof fin, hipMemcpyDeviceToHost);
    printf("%s: waiter %s, raiser %s, final %llu (expect %llu), marks", name, ok_b ? "done" : "STUCK", ok_a ? "done" : "STUCK",
           fin, base + 64ull * rounds);
    for (int r = 0; r < rounds; ++r) printf(" %u@%.3fms", h[r], r ? (w[r] - w[0]) / 1e5 : 0.0);
    printf("\n");
    return ok_a && ok_b ? 0 : 1;
}

int main() {
    unsigned long long *sig = nullptr;
    hipError_t e = hipExtMallocWithFlags((void **)&sig, sizeof(unsigned long long), hipMallocSignalMemory);
    printf("signal memory: %s\n", hipGetErrorString(e));
    int rc = 0;
    if (e == hipSuccess) rc |= probe("signal", sig);
    unsigned long long *dm = nullptr;
    (void)hipMalloc(&dm, 8);
    (void)hipMemset(dm, 0, 8);
    rc |= probe("device", dm) << 1;
    printf("rc %d\n", rc);
    return 0;
}
