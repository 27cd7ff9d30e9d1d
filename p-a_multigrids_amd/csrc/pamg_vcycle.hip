// Fused V-cycle for gfx950: one launch runs one pass of the n_multigrid loop
// body of transport_tri_semi.F90:319-379 for every un_ele.
//
// Every operation of the V-cycle is local to one unstructured element (the
// smoother, residual and RHS use the element's 3x3 operator; the children of a
// coarse sub-element live in the same un_ele, splitting.F90:97-140), so a
// workgroup can carry a tile of whole un_eles through the complete V-cycle
// without exchanging data with other workgroups. A tile holds 1024 level-1
// sub-elements (1024 / 4**(n_split-1) un_eles), 256 level-2 ones, 64 level-3
// ones, ...; 512 threads own two level-1 sub-elements each and one sub-element
// of every coarser level. The state between the steps lives in registers, the
// inter-level transfers go through LDS. HBM is touched once per field and
// level: tnew, RHS (level 1) and the previous residual are read, and tnew,
// tnew_nonlin (level 1), the new residual and the restricted RHS are written.
//
// The computation is the reference's, step for step and in its operation
// order (same device helpers as the per-step kernels; results are bitwise
// equal to pamg_vcycle's multi-kernel form, tests/test_gpu_parity.py):
//   restriction leg  l = 1..L : smoother (n sweeps, halo), restrictor of the
//                               previous residual, new residual   (:323-340)
//   coarsest level            : 15 smoother calls = 15 n sweeps   (:344-359)
//   prolongation leg l = L-1..1: prolongator (computed on chip; the reference
//                               overwrites its result with tnew_nonlin at the
//                               first sweep, :550), smoother      (:363-378)
// What is not written back is only what the reference overwrites before any
// read: the intermediate tnew of each level and the prolonged tnew.
#include <hip/hip_runtime.h>

#include "pamg_device.h"
#include "pamg_internal.h"

namespace pamg {
namespace {

using namespace detail;

constexpr int kMT = 512;    // threads per workgroup
constexpr int kT1 = 1024;   // level-1 sub-elements per tile

struct VLevel {
    double *T, *TNN, *RHS, *RES;
    const double *stc;
    const int4 *children;   // children (in-un_ele indices) of this level's sub-elements in the next finer level
    int64_t pitch;
    int nsub_log2;
    HaloArgs H;
};

struct VArgs {
    VLevel lv[kMaxFusedLevels];
    int64_t U;
    int G_log2;             // un_eles per tile = 1024 / nsub_1
    int n_smooth, n_coarse;
    double rdt;
};

struct Sub {
    double p[3], x[3], b[3];
};

__device__ __forceinline__ void load3(const double *f, int64_t pitch, int64_t s, double v[3]) {
#pragma unroll
    for (int c = 0; c < 3; ++c) v[c] = f[c * pitch + s];
}
__device__ __forceinline__ void store3(double *f, int64_t pitch, int64_t s, const double v[3]) {
#pragma unroll
    for (int c = 0; c < 3; ++c) f[c * pitch + s] = v[c];
}

// one smoother call (or several) on one sub-element: x -> last iterate, p -> iterate before the last sweep
__device__ __forceinline__ void smooth_sub(const VLevel &V, int64_t s, int sweeps, double rdt, Sub &q) {
    Stc S;
    load_stc(V.stc + (s >> V.nsub_log2) * kStcStride, S);
#pragma unroll
    for (int c = 0; c < 3; ++c) q.p[c] = q.x[c];
    for (int it = 0; it < sweeps; ++it) {
#pragma unroll
        for (int c = 0; c < 3; ++c) q.p[c] = q.x[c];
        sweep(S, rdt, q.b, q.x);
    }
}

// the halo words of one sub-element (update_overlaps at the start of the last sweep, :555)
__device__ __forceinline__ void halo_sub(const VLevel &V, int64_t s, const double t[3]) {
    const HaloArgs &H = V.H;
    const int4 hs = H.hsub[s & ((1ll << V.nsub_log2) - 1)];
    if ((hs.x | hs.y | hs.z) == 0) return;
    const int64_t u = s >> V.nsub_log2;
    const int4 r1 = H.hface[3 * u], r2 = H.hface[3 * u + 1], r3 = H.hface[3 * u + 2];
    int e = -1;
    if (hs.x && (r1.x & 3)) e = r1.w + hs.x - 1;
    else if (hs.y && (r2.x & 3)) e = r2.w + hs.y - 1;
    else if (hs.z && (r3.x & 3)) e = r3.w + hs.z - 1;
    double to[3] = {0.0, 0.0, 0.0};
    if (e >= 0) {
#pragma unroll
        for (int c = 0; c < 3; ++c) to[c] = H.told[3 * (int64_t)e + c];
    }
    if (hs.x) halo_face(H, r1, 1, hs.x, t, to);
    if (hs.y) halo_face(H, r2, 2, hs.y, t, to);
    if (hs.z) halo_face(H, r3, 3, hs.z, t, to);
}

__device__ __forceinline__ void residual_sub(const VLevel &V, int64_t s, double rdt, const Sub &q) {
    Stc S;
    load_stc(V.stc + (s >> V.nsub_log2) * kStcStride, S);
    double A[3], r[3];
    apply_A(S, rdt, q.p, A);
#pragma unroll
    for (int c = 0; c < 3; ++c) r[c] = A[c] - q.b[c];
    store3(V.RES, V.pitch, s, r);
}

// prolongator cascade (splitting.F90:59-88) on the LDS image of the fine tile
__device__ __forceinline__ void prolong_cascade(double *F, int nf, const int fi[4], const double y[3]) {
    double f[4][3];
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int i = 0; i < 3; ++i) f[q][i] = F[i * nf + fi[q]];
    f[0][0] = f[0][0] + 0.5 * y[2] + 0.5 * y[0];
    f[0][1] = f[0][1] + 0.5 * y[1] + 0.5 * y[2];
    f[0][2] = f[0][2] + y[2];
    f[1][0] = f[1][0] + f[0][1];
    f[1][1] = f[1][1] + f[0][0];
    f[1][2] = f[1][2] + 0.5 * y[0] + 0.5 * y[1];
    f[2][0] = f[2][0] + y[0];
    f[2][1] = f[2][1] + f[1][2];
    f[2][2] = f[2][2] + f[1][1];
    f[3][0] = f[3][0] + f[1][2];
    f[3][1] = f[3][1] + y[1];
    f[3][2] = f[3][2] + f[1][0];
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int i = 0; i < 3; ++i) F[i * nf + fi[q]] = f[q][i];
}

// Sub-element ownership inside a tile: level 1 -> tile-local t and t + 512,
// level l >= 2 -> t (if t < n_l). Per-level register state st[l][k].
template <int L>
__global__ __launch_bounds__(kMT) void k_vcycle(VArgs A) {
    __shared__ __attribute__((aligned(16))) double lds[3 * (kT1 + kT1 / 4)];
    const int t = threadIdx.x;
    const int64_t u0 = (int64_t)blockIdx.x << A.G_log2;                  // first un_ele of the tile
    const int64_t nue = min((int64_t)1 << A.G_log2, A.U - u0);          // un_eles in this tile
    const double rdt = A.rdt;
    Sub st[L][2];
    int nl[L];      // sub-elements of the tile on each level
    int64_t s0[L];  // first global sub-element of the tile on each level
#pragma unroll
    for (int l = 0; l < L; ++l) {
        nl[l] = (int)(nue << A.lv[l].nsub_log2);
        s0[l] = u0 << A.lv[l].nsub_log2;
    }
    // ---- restriction leg (:323-340)
#pragma unroll
    for (int l = 0; l < L; ++l) {
        const VLevel &V = A.lv[l];
        const int K = (l == 0) ? 2 : 1;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int j = t + k * kMT;
            if (j >= nl[l]) continue;
            const int64_t s = s0[l] + j;
            load3(V.T, V.pitch, s, st[l][k].x);                 // tnew_nonlin := tnew (:327)
            if (l == 0) load3(V.RHS, V.pitch, s, st[l][k].b);   // RHS_1 (get_RHS, constant in the step)
            smooth_sub(V, s, A.n_smooth, rdt, st[l][k]);       // call smoother (:331)
            halo_sub(V, s, st[l][k].p);
        }
        if (l + 1 < L) {                                        // call restrictor (:336)
            const VLevel &C = A.lv[l + 1];
            double *R = lds;
            for (int j = t; j < nl[l]; j += kMT) {
                double r[3];
                load3(V.RES, V.pitch, s0[l] + j, r);           // previous cycle's residual
#pragma unroll
                for (int c = 0; c < 3; ++c) R[c * nl[l] + j] = r[c];
            }
            __syncthreads();
            if (t < nl[l + 1]) {
                const int cin = t & ((1 << C.nsub_log2) - 1);
                const int base = (t >> C.nsub_log2) << V.nsub_log2;
                const int4 ch = C.children[cin];
                const int pick[3] = {base + ch.z, base + ch.w, base + ch.x};
#pragma unroll
                for (int i = 0; i < 3; ++i)
                    st[l + 1][0].b[i] = (R[pick[i]] + R[nl[l] + pick[i]] + R[2 * nl[l] + pick[i]]) / 3.;
                store3(C.RHS, C.pitch, s0[l + 1] + t, st[l + 1][0].b);
            }
            __syncthreads();
        }
#pragma unroll
        for (int k = 0; k < K; ++k) {                           // call get_residual (:338)
            const int j = t + k * kMT;
            if (j < nl[l]) residual_sub(V, s0[l] + j, rdt, st[l][k]);
        }
    }
    // ---- coarsest level: 15 smoother calls from tnew_nonlin := tnew (:344-359)
    {
        constexpr int l = L - 1;
        const VLevel &V = A.lv[l];
        const int K = (l == 0) ? 2 : 1;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int j = t + k * kMT;
            if (j >= nl[l]) continue;
            const int64_t s = s0[l] + j;
            Sub q = st[l][k];
#pragma unroll
            for (int c = 0; c < 3; ++c) q.x[c] = q.p[c];
            smooth_sub(V, s, A.n_smooth * A.n_coarse, rdt, q);
            halo_sub(V, s, q.p);
            store3(V.T, V.pitch, s, q.p);
            if (l == 0) store3(V.TNN, V.pitch, s, q.x);
            st[l][k].p[0] = q.p[0]; st[l][k].p[1] = q.p[1]; st[l][k].p[2] = q.p[2];   // final tnew of the level
        }
    }
    // ---- prolongation leg (:363-378)
#pragma unroll
    for (int l = L - 2; l >= 0; --l) {
        const VLevel &V = A.lv[l], &C = A.lv[l + 1];
        const int K = (l == 0) ? 2 : 1;
        double *F = lds, *Y = lds + 3 * nl[l];
        // prolongator (:370) on the LDS image of tnew (= tnew_nonlin, :367) with the final coarse tnew
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int j = t + k * kMT;
            if (j < nl[l])
#pragma unroll
                for (int c = 0; c < 3; ++c) F[c * nl[l] + j] = st[l][k].p[c];
        }
        if (t < nl[l + 1])
#pragma unroll
            for (int c = 0; c < 3; ++c) Y[c * nl[l + 1] + t] = st[l + 1][0].p[c];
        __syncthreads();
        if (t < nl[l + 1]) {
            const int cin = t & ((1 << C.nsub_log2) - 1);
            const int base = (t >> C.nsub_log2) << V.nsub_log2;
            const int4 ch = C.children[cin];
            const int fi[4] = {base + ch.x, base + ch.y, base + ch.z, base + ch.w};
            const double y[3] = {Y[t], Y[nl[l + 1] + t], Y[2 * nl[l + 1] + t]};
            prolong_cascade(F, nl[l], fi, y);
        }
        __syncthreads();
        // smoother from tnew_nonlin (:376): the prolonged tnew is overwritten at its first sweep (:550)
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int j = t + k * kMT;
            if (j >= nl[l]) continue;
            const int64_t s = s0[l] + j;
            Sub q = st[l][k];
#pragma unroll
            for (int c = 0; c < 3; ++c) q.x[c] = q.p[c];
            smooth_sub(V, s, A.n_smooth, rdt, q);
            halo_sub(V, s, q.p);
            store3(V.T, V.pitch, s, q.p);
            if (l == 0) store3(V.TNN, V.pitch, s, q.x);
            st[l][k].p[0] = q.p[0]; st[l][k].p[1] = q.p[1]; st[l][k].p[2] = q.p[2];
        }
    }
}

}  // namespace

bool vcycle_fusable(const Level *lv, int L, int n_split, int solver, int halo_mode, int n_smooth) {
    (void)lv;
    return solver != 2 && halo_mode == 0 && n_smooth > 0 && L >= 1 && L <= kMaxFusedLevels && n_split <= 5 &&
           n_split >= L;
}

hipError_t launch_vcycle(hipStream_t s, const Level *lv, int L, int U, int n_split, int n_smooth, int n_coarse,
                         double rdt, double *tov, double *tovo) {
    VArgs A{};
    for (int l = 0; l < L; ++l) {
        const Level &V = lv[l + 1];
        VLevel &o = A.lv[l];
        o.T = V.T; o.TNN = V.TNN; o.RHS = V.RHS; o.RES = V.RES; o.stc = V.stc;
        o.children = (l > 0) ? lv[l].children : nullptr;   // children of level l+1 in level l
        o.pitch = V.pitch;
        int lg = 0;
        while ((1 << lg) < V.nsub) ++lg;
        o.nsub_log2 = lg;
        const HaloPlan &P = V.halo;
        o.H = HaloArgs{P.d_hsub, P.d_hface, P.d_bcv, P.d_told_halo, tov, tovo, P.d_send, 1 << V.isplit};
    }
    A.U = U;
    A.G_log2 = 10 - 2 * n_split;   // 1024 / 4**n_split un_eles per tile
    A.n_smooth = n_smooth;
    A.n_coarse = n_coarse;
    A.rdt = rdt;
    const unsigned grid = (unsigned)((U + (1 << A.G_log2) - 1) >> A.G_log2);
    if (grid == 0) return hipSuccess;
    switch (L) {
        case 1: hipLaunchKernelGGL(k_vcycle<1>, dim3(grid), dim3(kMT), 0, s, A); break;
        case 2: hipLaunchKernelGGL(k_vcycle<2>, dim3(grid), dim3(kMT), 0, s, A); break;
        case 3: hipLaunchKernelGGL(k_vcycle<3>, dim3(grid), dim3(kMT), 0, s, A); break;
        case 4: hipLaunchKernelGGL(k_vcycle<4>, dim3(grid), dim3(kMT), 0, s, A); break;
        case 5: hipLaunchKernelGGL(k_vcycle<5>, dim3(grid), dim3(kMT), 0, s, A); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace pamg
