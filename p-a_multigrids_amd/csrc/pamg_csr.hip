// The matrices.F90 SpMV: csr_mul_array (matrices.F90:172-193) on the device, over the
// reference's own `type sparse` storage (Structures.F90:196-201).
//
// The reference walks the entries in storage order, three per row, for size(g_iloc) rows
// (it never reads g_iloc's values: every row of its matrices holds the same number of
// entries, and a 9-per-row flux matrix would be read as if it had 3), starting each row at
// 0 and accumulating val(c) * array(g_jloc(c)) -- one row per thread here, the same
// products and additions in the same order without contraction: bitwise equal to the
// reference (tests/test_csr.py). HBM-bound gather SpMV: 3 x (4 B column + 8 B value) +
// 8 B result per row, plus the gathered array; the entries are streamed once with
// non-temporal loads.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <string>
#include <vector>

#include "pamg_internal.h"

struct pamg_csr {
    int device = 0;
    long nrows = 0, nnz = 0;
    int max_col = 0;          // largest 1-based column: the array must hold at least this many
    int *jloc = nullptr;      // g_jloc, 1-based, first 3 nrows entries (the ones the routine reads)
    double *val = nullptr;
    double *x = nullptr, *y = nullptr;   // device staging of array / result (host-pointer calls)
    long x_cap = 0;
};

namespace {

constexpr int kCsrBlock = 256;

__global__ __launch_bounds__(kCsrBlock) void k_csr_mul_array(const int *__restrict__ jloc,
                                                             const double *__restrict__ val,
                                                             const double *__restrict__ x,
                                                             double *__restrict__ y, long nrows) {
    const long r = (long)blockIdx.x * kCsrBlock + threadIdx.x;
    if (r >= nrows) return;
    const long c = 3 * r;
    double acc = 0.0;   // result = 0.0 (:186); 0.0 + v*a keeps the reference's signed zero
#pragma unroll
    for (int n = 0; n < 3; ++n) {
        const int j = __builtin_nontemporal_load(jloc + c + n);
        const double v = __builtin_nontemporal_load(val + c + n);
        acc = acc + v * x[j - 1];
    }
    y[r] = acc;
}

int fail(pamg_handle *h, hipError_t e, const char *what) {
    if (h) h->err = std::string(what) + ": " + hipGetErrorString(e);
    return PAMG_ERR_HIP;
}

}  // namespace

extern "C" {

int pamg_csr_create(pamg_handle *h, long nrows, long nnz, const int *g_jloc, const double *val, pamg_csr **out) {
    if (!h || !out || !g_jloc || !val || nrows < 1 || nnz < 3 * nrows) {
        if (h) h->err = "pamg_csr_create: csr_mul_array reads 3 entries per row: need nnz >= 3 nrows >= 3";
        return PAMG_ERR_ARG;
    }
    *out = nullptr;
    const long used = 3 * nrows;
    int mx = 0;
    for (long c = 0; c < used; ++c) {
        if (g_jloc[c] < 1) { h->err = "pamg_csr_create: g_jloc entries are 1-based"; return PAMG_ERR_ARG; }
        mx = std::max(mx, g_jloc[c]);
    }
    auto *m = new pamg_csr;
    m->device = h->device;
    m->nrows = nrows;
    m->nnz = nnz;
    m->max_col = mx;
    hipError_t e;
    if ((e = hipSetDevice(h->device)) != hipSuccess || (e = hipMalloc(&m->jloc, used * sizeof(int))) != hipSuccess ||
        (e = hipMalloc(&m->val, used * sizeof(double))) != hipSuccess ||
        (e = hipMemcpyAsync(m->jloc, g_jloc, used * sizeof(int), hipMemcpyHostToDevice, h->stream)) != hipSuccess ||
        (e = hipMemcpyAsync(m->val, val, used * sizeof(double), hipMemcpyHostToDevice, h->stream)) != hipSuccess ||
        (e = hipStreamSynchronize(h->stream)) != hipSuccess) {   // on h's stream, as the SpMV that reads them
        pamg_csr_free(m);
        return fail(h, e, "pamg_csr_create");
    }
    *out = m;
    return PAMG_OK;
}

// device pointers: d_array holds >= max_col values, d_result nrows values (on h's stream)
int pamg_csr_mul_array_device(pamg_handle *h, pamg_csr *m, long n, const double *d_array, double *d_result) {
    if (!h || !m || !d_array || !d_result) return PAMG_ERR_ARG;
    if (n < m->max_col) { h->err = "csr_mul_array: array shorter than the largest column"; return PAMG_ERR_ARG; }
    const unsigned grid = (unsigned)((m->nrows + kCsrBlock - 1) / kCsrBlock);
    hipLaunchKernelGGL(k_csr_mul_array, dim3(grid), dim3(kCsrBlock), 0, h->stream, m->jloc, m->val, d_array,
                       d_result, m->nrows);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? PAMG_OK : fail(h, e, "k_csr_mul_array");
}

int pamg_csr_mul_array(pamg_handle *h, pamg_csr *m, long n, const double *array, double *result) {
    if (!h || !m || !array || !result) return PAMG_ERR_ARG;
    if (n < m->max_col) { h->err = "csr_mul_array: array shorter than the largest column"; return PAMG_ERR_ARG; }
    hipError_t e;
    if (n > m->x_cap) {
        (void)hipFree(m->x);
        m->x = nullptr;
        m->x_cap = 0;
        if ((e = hipMalloc(&m->x, n * sizeof(double))) != hipSuccess) return fail(h, e, "csr_mul_array");
        m->x_cap = n;
    }
    if (!m->y && (e = hipMalloc(&m->y, m->nrows * sizeof(double))) != hipSuccess) return fail(h, e, "csr_mul_array");
    if ((e = hipMemcpyAsync(m->x, array, n * sizeof(double), hipMemcpyHostToDevice, h->stream)) != hipSuccess)
        return fail(h, e, "csr_mul_array");
    const int rc = pamg_csr_mul_array_device(h, m, n, m->x, m->y);
    if (rc != PAMG_OK) return rc;
    if ((e = hipMemcpyAsync(result, m->y, m->nrows * sizeof(double), hipMemcpyDeviceToHost, h->stream)) !=
            hipSuccess ||
        (e = hipStreamSynchronize(h->stream)) != hipSuccess)
        return fail(h, e, "csr_mul_array");
    return PAMG_OK;
}

// roofline measurement: `reps` launches on device vectors (array = n values filled with 1),
// average launch time from HIP events on the handle's stream
int pamg_csr_bench(pamg_handle *h, pamg_csr *m, long n, int reps, double *ms_avg) {
    if (!h || !m || !ms_avg || reps < 1 || n < m->max_col) return PAMG_ERR_ARG;
    double *x = nullptr, *y = nullptr;
    hipEvent_t a = nullptr, b = nullptr;
    hipError_t e;
    int rc = PAMG_OK;
    if ((e = hipMalloc(&x, n * sizeof(double))) != hipSuccess || (e = hipMalloc(&y, m->nrows * sizeof(double))) != hipSuccess ||
        (e = hipMemsetAsync(x, 0, n * sizeof(double), h->stream)) != hipSuccess ||
        (e = hipEventCreate(&a)) != hipSuccess || (e = hipEventCreate(&b)) != hipSuccess) {
        rc = fail(h, e, "pamg_csr_bench");
    } else {
        rc = pamg_csr_mul_array_device(h, m, n, x, y);   // warm-up
        if (rc == PAMG_OK && (e = hipEventRecord(a, h->stream)) != hipSuccess) rc = fail(h, e, "pamg_csr_bench");
        for (int r = 0; r < reps && rc == PAMG_OK; ++r) rc = pamg_csr_mul_array_device(h, m, n, x, y);
        float ms = 0.f;
        if (rc == PAMG_OK && ((e = hipEventRecord(b, h->stream)) != hipSuccess || (e = hipEventSynchronize(b)) != hipSuccess ||
                              (e = hipEventElapsedTime(&ms, a, b)) != hipSuccess))
            rc = fail(h, e, "pamg_csr_bench");
        *ms_avg = ms / reps;
    }
    if (a) (void)hipEventDestroy(a);
    if (b) (void)hipEventDestroy(b);
    if (x) (void)hipFree(x);
    if (y) (void)hipFree(y);
    return rc;
}

int pamg_csr_free(pamg_csr *m) {
    if (!m) return PAMG_OK;
    (void)hipSetDevice(m->device);
    for (void *p : {(void *)m->jloc, (void *)m->val, (void *)m->x, (void *)m->y})
        if (p) (void)hipFree(p);
    delete m;
    return PAMG_OK;
}

}  // extern "C"
