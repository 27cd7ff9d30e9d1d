// Fused V-cycle for gfx950: two launches run one pass of the n_multigrid
// loop body of transport_tri_semi.F90:319-379 for every un_ele.
//
// Every operation of the V-cycle is local to one unstructured element (the
// smoother, residual and RHS use the element's 3x3 operator; the children of a
// coarse sub-element live in the same un_ele, splitting.F90:97-140), so a
// workgroup carries a tile of whole un_eles through its part of the cycle
// without exchanging data with other workgroups. The computation is the
// reference's, step for step and in its operation order (same device helpers
// as the per-step kernels; results are bitwise equal to pamg_vcycle's
// multi-kernel form, tests/test_gpu_parity.py). The schedule follows the data
// dependences, which the block-diagonal operator leaves loose:
//   * the restrictor (:336) reads the residual of the PREVIOUS cycle;
//   * the prolongation-leg smoother of level l (:376) starts from
//     tnew_nonlin = the restriction-leg tnew of level l (:367); the prolonged
//     values are overwritten at its first sweep (:550);
//   * so level 1 (the reference's finest level) depends on the coarser levels
//     only through the prolongator's (dead) result and the halo words, whose
//     final state is what level 1's last smoother call writes.
// Launch 1, k_vc_coarse: levels 2..L of the cycle -- all restrictions (level
//   1's from the old residual), both legs of every coarser level, the 15
//   coarse smoother calls, the prolongator cascades among them. Small
//   workgroups (256 level-2 sub-elements per tile): the 15 n_smooth dependent
//   sweeps of the coarsest level are a latency chain, hidden by occupancy.
// Launch 2, k_vc_fine: level 1 -- both smoother calls, get_residual, and the
//   prolongator cascade from the final level-2 tnew; a streaming kernel
//   (tnew, RHS in; residual, tnew, tnew_nonlin out) whose halo words are the
//   cycle's last, as in the reference.
// Levels are 0-based inside this file: level 0 = the reference's level 1.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <type_traits>
#include <vector>

#include "pamg_device.h"
#include "pamg_internal.h"

namespace pamg {
namespace {

using namespace detail;

constexpr int kMTf = 512;   // threads per workgroup, level-0 kernel (one adjacent pair each)
constexpr int kMTc = 64;    // threads per workgroup, coarse-level kernel (one wave per tile)

struct VLevel {
    double *T, *TNN, *RHS, *RES;
    const double *stc;
    const int4 *children;   // children (in-un_ele indices) of this level's sub-elements in the next finer level
    int64_t pitch;
    HaloArgs H;
};

struct VArgs {
    VLevel lv[kMaxFusedLevels];
    int64_t U;
    int n_smooth, n_coarse;
    double rdt;
    int cascade;            // 0: skip the (dead) prolongator cascades (PAMG_DIAG_NOCASCADE diagnostics)
    long long *stamps;      // phase timeline (PAMG_VCYCLE_STAMPS diagnostics), null otherwise
};

// phase stamps: 100 MHz wall clock per wave at the phase boundaries, plus the wave's HW_ID
constexpr int kStampSlots = 10;
template <int MT>
__device__ __forceinline__ void stamp(const VArgs &A, int i) {
    if (A.stamps && (threadIdx.x & 63) == 0)
        A.stamps[((int64_t)blockIdx.x * (MT / 64) + (threadIdx.x >> 6)) * kStampSlots + i] = wall_clock64();
}
template <int MT>
__device__ __forceinline__ void stamp_hwid(const VArgs &A) {
    if (A.stamps && (threadIdx.x & 63) == 0) {
        unsigned hw;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        A.stamps[((int64_t)blockIdx.x * (MT / 64) + (threadIdx.x >> 6)) * kStampSlots + 9] = hw;
    }
}

// tile geometry (0-based level l): 4**(S-l) sub-elements per un_ele; a tile holds
// 1024 >> 2l sub-elements of level l (1024 / 4**S un_eles)
template <int S, int L>
struct Geo {
    static constexpr int C = L - 1;                                // coarsest level
    static constexpr int GL = 10 - 2 * S;                          // log2 un_eles per tile
    static constexpr int lg(int l) { return 2 * (S - l); }
    static constexpr int nt(int l) { return 1024 >> (2 * l); }
    // each wave inside one un_ele (a wave spans 128 level-0 sub-elements, 64 of any other level)
    static constexpr bool uni(int l) { return lg(l) >= (l == 0 ? 7 : 6); }
};

// field access: wave-uniform plane base (SGPRs) + 32-bit sub-element index (one VGPR for all planes)
__device__ __forceinline__ void load3(const double *f, int64_t pitch, uint32_t s, double v[3]) {
    const uint32_t o = s << 3;
#pragma unroll
    for (int c = 0; c < 3; ++c) v[c] = *reinterpret_cast<const double *>(reinterpret_cast<const char *>(f + c * pitch) + o);
}
__device__ __forceinline__ void store3(double *f, int64_t pitch, uint32_t s, const double v[3]) {
    const uint32_t o = s << 3;
#pragma unroll
    for (int c = 0; c < 3; ++c) *reinterpret_cast<double *>(reinterpret_cast<char *>(f + c * pitch) + o) = v[c];
}
// the adjacent pair s, s+1 (s even) with 16-byte accesses
__device__ __forceinline__ void load3p(const double *f, int64_t pitch, uint32_t s, double a[3], double b[3]) {
    const uint32_t o = s << 3;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        const double2 v = *reinterpret_cast<const double2 *>(reinterpret_cast<const char *>(f + c * pitch) + o);
        a[c] = v.x;
        b[c] = v.y;
    }
}
__device__ __forceinline__ void store3p(double *f, int64_t pitch, uint32_t s, const double a[3], const double b[3]) {
    const uint32_t o = s << 3;
#pragma unroll
    for (int c = 0; c < 3; ++c)
        *reinterpret_cast<double2 *>(reinterpret_cast<char *>(f + c * pitch) + o) = make_double2(a[c], b[c]);
}
__device__ __forceinline__ void copy3(double d[3], const double s[3]) {
#pragma unroll
    for (int c = 0; c < 3; ++c) d[c] = s[c];
}

template <int I, int N, class F>
__device__ __forceinline__ void static_for(F &&f) {
    if constexpr (I < N) {
        f(std::integral_constant<int, I>{});
        static_for<I + 1, N>(f);
    }
}

// operator record of un_ele u; wave-uniform records come through the scalar cache
// (uni is a compile-time constant at every call site once the level loops are unrolled)
__device__ __forceinline__ void stencil(bool uni, const double *__restrict__ stc, uint32_t u, Stc &S) {
    if (uni) u = __builtin_amdgcn_readfirstlane(u);
    load_stc(stc + u * (uint32_t)kStcStride, S);
}

// n sweeps from x: x -> last iterate, p -> iterate before the last sweep (n >= 1)
__device__ __forceinline__ void sweeps(const Stc &S, double rdt, int n, const double b[3], double x[3],
                                       double p[3]) {
    for (int it = 0; it < n; ++it) {
        copy3(p, x);
        sweep(S, rdt, b, x);
    }
}
// two sub-elements of one un_ele, interleaved
__device__ __forceinline__ void sweeps2(const Stc &S, double rdt, int n, const double b0[3], const double b1[3],
                                        double x0[3], double x1[3], double p0[3], double p1[3]) {
    for (int it = 0; it < n; ++it) {
        copy3(p0, x0);
        copy3(p1, x1);
        sweep(S, rdt, b0, x0);
        sweep(S, rdt, b1, x1);
    }
}

// N sub-elements of one un_ele, interleaved
template <int N>
__device__ __forceinline__ void sweepsN(const Stc &S, double rdt, int n, const double b[N][3], double x[N][3],
                                        double p[N][3]) {
    for (int it = 0; it < n; ++it) {
#pragma unroll
        for (int q = 0; q < N; ++q) copy3(p[q], x[q]);
#pragma unroll
        for (int q = 0; q < N; ++q) sweep(S, rdt, b[q], x[q]);
    }
}

__device__ __forceinline__ void residual(const Stc &S, double rdt, const double p[3], const double b[3],
                                         double r[3]) {
    double a[3];
    apply_A(S, rdt, p, a);
#pragma unroll
    for (int c = 0; c < 3; ++c) r[c] = a[c] - b[c];
}

// ---- halo words of one sub-element (update_overlaps, :555)
// h: its positions along faces 1..3 packed 6 bits each (0: not on that face)
__device__ __forceinline__ int hs_pack(int4 q) { return q.x | (q.y << 6) | (q.z << 12); }

// tnew words of the halo (update_overlaps); t_overlap_old and the boundary values are
// constant within a time step and are written by k_overlap_static (pamg_kernels.hip)
__device__ __forceinline__ void hs_write(bool uni, const HaloArgs &H, uint32_t u, int h, const double t[3]) {
    if (h == 0) return;
    if (uni) u = __builtin_amdgcn_readfirstlane(u);
    const int4 r1 = H.hface[3 * u], r2 = H.hface[3 * u + 1], r3 = H.hface[3 * u + 2];
    const int a = h & 63, b = (h >> 6) & 63, c = h >> 12;
    if (a) halo_face<true, false>(H, r1, 1, a, t, t);
    if (b) halo_face<true, false>(H, r2, 2, b, t, t);
    if (c) halo_face<true, false>(H, r3, 3, c, t, t);
}

// prolongator cascade (splitting.F90:59-88) on the LDS image of the fine tile (component stride n)
__device__ __forceinline__ void prolong_cascade(double *F, int n, const int fi[4], const double y[3]) {
    double f[4][3];
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int i = 0; i < 3; ++i) f[q][i] = F[i * n + fi[q]];
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
        for (int i = 0; i < 3; ++i) F[i * n + fi[q]] = f[q][i];
}

// ===================================================================== coarse levels
// One wave per tile. Level l >= 1 of a tile has nt(l) sub-elements; lane t owns the
// sub-elements t + 64 k, k < K(l) = max(1, nt(l) / 64), that are < nt(l): four of
// level 1, one of level 2, one on the first nt(l) lanes below. The coarsest level's
// 1 + n_coarse smoother calls are a chain of dependent sweeps, issue-bound on the
// wave that runs it; with one wave per tile no wave waits on it, and the many tiles
// resident per CU overlap their memory phases with the chains of the others.
// LDS per level l: B_l = RHS (3 x nt(l)), W_l = tnew: the restriction-leg iterate
// (l < C) or, on the coarsest level, its tnew, and Y_l (2 <= l < C) the final tnew of
// a middle level (input of the prolongator cascade into level l - 1).
template <int S, int L>
struct CGeo {
    using G = Geo<S, L>;
    static constexpr int C = G::C;
    static constexpr int K(int l) { return G::nt(l) >= 64 ? G::nt(l) / 64 : 1; }
    // every lane of a chunk inside one un_ele (operator records through the scalar cache)
    static constexpr bool uni(int l) { return (G::nt(l) < 64 ? G::nt(l) : 64) <= (1 << G::lg(l)); }
    // every chunk of the level inside one un_ele: the chunks are smoothed together (ILP)
    static constexpr bool one(int l) { return G::nt(l) <= (1 << G::lg(l)); }
    static constexpr int sz(int l) { return 3 * G::nt(l); }
    static constexpr int B(int l) {
        int o = 0;
        for (int i = 1; i < l; ++i) o += 2 * sz(i);
        return o;
    }
    static constexpr int W(int l) { return B(l) + sz(l); }
    static constexpr int Y(int l) {   // 2 <= l < C
        int o = B(C + 1);
        for (int i = 2; i < l; ++i) o += sz(i);
        return o;
    }
    static constexpr int dump = Y(C);            // 3 slots per lane for the stores of idle lanes
    static constexpr int total = dump + 3 * 64;
    // restrictor chunks: (level l + 1, chunk k) for l = 0..C-1
    static constexpr int nrc() {
        int n = 0;
        for (int l = 1; l <= C; ++l) n += K(l);
        return n;
    }
};

template <int S, int L>
__global__ __launch_bounds__(kMTc) void k_vc_coarse(VArgs A, const double *__restrict__ sp1,
                                                    const double *__restrict__ sp2, const double *__restrict__ sp3,
                                                    const double *__restrict__ sp4) {
    // operator records as restrict kernel arguments: never written here, so wave-uniform
    // records are fetched with scalar loads
    const double *__restrict__ SP[kMaxFusedLevels] = {nullptr, sp1, sp2, sp3, sp4};
    using G = Geo<S, L>;
    using Q = CGeo<S, L>;
    constexpr int C = G::C;
    static_assert(C >= 1, "coarse kernel needs two levels");
    __shared__ __attribute__((aligned(16))) double lds[Q::total];
    const int t = threadIdx.x;
    const double rdt = A.rdt;
    const int ns = A.n_smooth;
    const int64_t u0 = (int64_t)blockIdx.x << G::GL;
    const int nue = (int)min((int64_t)1 << G::GL, A.U - u0);
    stamp<kMTc>(A, 0);
    stamp_hwid<kMTc>(A);
    // chunk k of level l: tile index t + 64 k, valid if inside the tile's un_eles; idle
    // lanes load index 0 (in bounds) and store to the dump slots (no branches, so the
    // loads of a phase are all in flight together)
    auto ok = [&](int l, int k) -> bool { return t + 64 * k < G::nt(l) && t + 64 * k < (nue << G::lg(l)); };
    auto gix = [&](int l, int k) -> uint32_t {
        return ((uint32_t)u0 << G::lg(l)) + (uint32_t)(ok(l, k) ? t + 64 * k : 0);
    };
    auto lix = [&](int base, int l, int k, int c) -> int {   // LDS slot of component c
        return ok(l, k) ? base + c * G::nt(l) + t + 64 * k : Q::dump + 3 * t + c;
    };
    // ---- prologue, batch 1: tnew of every level (tnew_nonlin := tnew, :327 / :348), halo
    //      positions, children of the restrictor chunks
    int hl[L][4];
    double xi[L][4][3];
    int4 ch[L][4];
#pragma unroll
    for (int l = 1; l < L; ++l)
#pragma unroll
        for (int k = 0; k < Q::K(l); ++k) {
            const uint32_t g = gix(l, k);
            load3(A.lv[l].T, A.lv[l].pitch, g, xi[l][k]);
            const int4 hs = A.lv[l].H.hsub[g & ((1 << G::lg(l)) - 1)];
            hl[l][k] = ok(l, k) ? hs_pack(hs) : 0;
            ch[l][k] = A.lv[l].children[g & ((1 << G::lg(l)) - 1)];
        }
#pragma unroll
    for (int l = 1; l < L; ++l)
#pragma unroll
        for (int k = 0; k < Q::K(l); ++k)
#pragma unroll
            for (int c = 0; c < 3; ++c) lds[lix(Q::W(l), l, k, c)] = xi[l][k][c];
    // ---- batch 2: restrictor (:336) of every level from the residual of the PREVIOUS cycle,
    //      RHS_{l+1}(1, c) = mean(res_l(:, f3)), (2, c) = mean(res_l(:, f4)), (3, c) = mean(res_l(:, f1))
    //      (splitting.F90:10-32, 146-151); all read before any residual is rewritten
    double rr[L][4][3][3];
#pragma unroll
    for (int l = 0; l < C; ++l)
#pragma unroll
        for (int k = 0; k < Q::K(l + 1); ++k) {
            const uint32_t g = gix(l + 1, k);
            const int4 c4 = ch[l + 1][k];
            const uint32_t base = (g >> G::lg(l + 1)) << G::lg(l);
            const uint32_t pick[3] = {base + c4.z, base + c4.w, base + c4.x};
#pragma unroll
            for (int q = 0; q < 3; ++q) load3(A.lv[l].RES, A.lv[l].pitch, pick[q], rr[l + 1][k][q]);
        }
#pragma unroll
    for (int l = 1; l <= C; ++l)
#pragma unroll
        for (int k = 0; k < Q::K(l); ++k) {
            double b[3];
#pragma unroll
            for (int q = 0; q < 3; ++q) b[q] = (rr[l][k][q][0] + rr[l][k][q][1] + rr[l][k][q][2]) / 3.;
            if (ok(l, k)) store3(A.lv[l].RHS, A.lv[l].pitch, gix(l, k), b);
#pragma unroll
            for (int c = 0; c < 3; ++c) lds[lix(Q::B(l), l, k, c)] = b[c];
        }
    stamp<kMTc>(A, 1);
    // smoother calls on the chunks of level l (x from W, b from B); the chunks of one un_ele
    // are interleaved (ILP), otherwise each reads its own operator record
    auto smooth_chunks = [&](auto LC, int nsw, double (&x)[4][3], const double (&b)[4][3], double (&p)[4][3]) {
        constexpr int l = decltype(LC)::value;
        constexpr int K = Q::K(l);
        if constexpr (Q::one(l)) {
            Stc St;
            stencil(Q::uni(l), SP[l], gix(l, 0) >> G::lg(l), St);
            sweepsN<K>(St, rdt, nsw, reinterpret_cast<const double(&)[K][3]>(b),
                       reinterpret_cast<double(&)[K][3]>(x), reinterpret_cast<double(&)[K][3]>(p));
        } else {
#pragma unroll
            for (int k = 0; k < K; ++k) {
                Stc St;
                stencil(Q::uni(l), SP[l], gix(l, k) >> G::lg(l), St);
                sweeps(St, rdt, nsw, b[k], x[k], p[k]);
            }
        }
    };
    auto residual_chunks = [&](auto LC, const double (&b)[4][3], const double (&p)[4][3]) {
        constexpr int l = decltype(LC)::value;
        const VLevel &V = A.lv[l];
#pragma unroll
        for (int k = 0; k < Q::K(l); ++k) {
            Stc St;
            stencil(Q::uni(l), SP[l], gix(l, k) >> G::lg(l), St);
            double r[3];
            residual(St, rdt, p[k], b[k], r);
            if (ok(l, k)) store3(V.RES, V.pitch, gix(l, k), r);
        }
    };
    auto load_wb = [&](auto LC, double (&x)[4][3], double (&b)[4][3]) {
        constexpr int l = decltype(LC)::value;
#pragma unroll
        for (int k = 0; k < Q::K(l); ++k)
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                x[k][c] = lds[lix(Q::W(l), l, k, c)];
                b[k][c] = lds[lix(Q::B(l), l, k, c)];
            }
    };
    auto halo_chunks = [&](auto LC, const double (&p)[4][3]) {
        constexpr int l = decltype(LC)::value;
#pragma unroll
        for (int k = 0; k < Q::K(l); ++k) hs_write(Q::uni(l), A.lv[l].H, gix(l, k) >> G::lg(l), hl[l][k], p[k]);
    };
    // ---- levels 1..C-1, restriction leg: smoother (:331), get_residual (:338)
    static_for<1, C>([&](auto LC) {
        constexpr int l = decltype(LC)::value;
        double x[4][3], b[4][3], p[4][3];
        load_wb(LC, x, b);
        smooth_chunks(LC, ns, x, b, p);
#pragma unroll
        for (int k = 0; k < Q::K(l); ++k)
#pragma unroll
            for (int c = 0; c < 3; ++c) lds[lix(Q::W(l), l, k, c)] = p[k][c];
        halo_chunks(LC, p);
        residual_chunks(LC, b, p);
    });
    stamp<kMTc>(A, 2);
    // ---- coarsest level: smoother + get_residual of the restriction leg, then the
    //      n_coarse smoother calls from tnew_nonlin := tnew (:344-359)
    {
        using LC = std::integral_constant<int, C>;
        double x[4][3], b[4][3], p[4][3];
        load_wb(LC{}, x, b);
        smooth_chunks(LC{}, ns, x, b, p);
        halo_chunks(LC{}, p);
        residual_chunks(LC{}, b, p);
#pragma unroll
        for (int k = 0; k < Q::K(C); ++k) copy3(x[k], p[k]);
        smooth_chunks(LC{}, ns * A.n_coarse, x, b, p);
        halo_chunks(LC{}, p);
#pragma unroll
        for (int k = 0; k < Q::K(C); ++k) {
            if (ok(C, k)) store3(A.lv[C].T, A.lv[C].pitch, gix(C, k), p[k]);
#pragma unroll
            for (int c = 0; c < 3; ++c) lds[lix(Q::W(C), C, k, c)] = p[k][c];
        }
    }
    stamp<kMTc>(A, 3);
    // ---- prolongation leg, levels C-1..1: smoother from tnew_nonlin = restriction-leg tnew (:367, :376)
    static_for<1, C>([&](auto LR) {
        constexpr int l = C - decltype(LR)::value;
        using LC = std::integral_constant<int, l>;
        double x[4][3], b[4][3], p[4][3];
        load_wb(LC{}, x, b);
        smooth_chunks(LC{}, ns, x, b, p);
        halo_chunks(LC{}, p);
#pragma unroll
        for (int k = 0; k < Q::K(l); ++k) {
            if (ok(l, k)) store3(A.lv[l].T, A.lv[l].pitch, gix(l, k), p[k]);
            if constexpr (l >= 2)
#pragma unroll
                for (int c = 0; c < 3; ++c) lds[lix(Q::Y(l), l, k, c)] = p[k][c];
        }
    });
    stamp<kMTc>(A, 4);
    // ---- prolongator (:370) among the coarse levels, on the LDS images of the
    //      restriction-leg tnew (its result is dead, :550)
    if constexpr (C >= 2) {
        __syncthreads();
#pragma unroll
        for (int l = 1; l < C; ++l) {
            const int ysrc = (l + 1 == C) ? Q::W(C) : Q::Y(l + 1);
#pragma unroll
            for (int k = 0; k < Q::K(l + 1); ++k) {
                if (!ok(l + 1, k)) continue;
                const int j = t + 64 * k;
                const int4 c4 = ch[l + 1][k];
                const int base = (j >> G::lg(l + 1)) << G::lg(l);
                const int fi[4] = {base + c4.x, base + c4.y, base + c4.z, base + c4.w};
                const double y[3] = {lds[ysrc + j], lds[ysrc + G::nt(l + 1) + j], lds[ysrc + 2 * G::nt(l + 1) + j]};
                prolong_cascade(lds + Q::W(l), G::nt(l), fi, y);
            }
            __syncthreads();
        }
    }
    stamp<kMTc>(A, 7);
}

// ===================================================================== level 0
// Ownership: the adjacent pair 2t, 2t+1 of the tile (16-byte accesses, one un_ele,
// one operator record); for the prolongator, level-1 sub-element t.
template <int S, int L>
__global__ __launch_bounds__(kMTf, (S >= 3) ? 4 : 2) void k_vc_fine(VArgs A, const double *__restrict__ sp0) {
    using G = Geo<S, L>;
    constexpr int C = G::C;
    __shared__ __attribute__((aligned(16))) double F0[C > 0 ? 3 * 1024 : 1];   // restriction-leg tnew image
    const int t = threadIdx.x;
    const double rdt = A.rdt;
    const int ns = A.n_smooth;
    const int64_t u0 = (int64_t)blockIdx.x << G::GL;
    const int nue = (int)min((int64_t)1 << G::GL, A.U - u0);
    stamp<kMTf>(A, 0);
    stamp_hwid<kMTf>(A);
    const VLevel &V0 = A.lv[0];
    const bool v0 = 2 * t < (nue << G::lg(0));
    const uint32_t s0 = ((uint32_t)u0 << G::lg(0)) + (v0 ? 2 * t : 0);   // clamped: loads stay in bounds
    const uint32_t w0 = s0 >> G::lg(0);                                  // un_ele of the pair
    // ---- prologue
    int h0[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) h0[k] = v0 ? hs_pack(V0.H.hsub[(s0 + k) & ((1 << G::lg(0)) - 1)]) : 0;
    double x0[2][3], b0[2][3], p0[2][3];
    load3p(V0.T, V0.pitch, s0, x0[0], x0[1]);      // tnew_nonlin := tnew (:327)
    load3p(V0.RHS, V0.pitch, s0, b0[0], b0[1]);    // RHS of level 1 (get_RHS, constant in the time step)
    // final level-1 tnew (coarse launch) for the prolongator
    bool v1 = false;
    uint32_t s1 = 0;
    double y1[3];
    int4 c4 = make_int4(0, 0, 0, 0);
    if constexpr (C > 0) {
        v1 = t < (nue << G::lg(1));
        s1 = ((uint32_t)u0 << G::lg(1)) + (v1 ? t : 0);
        load3(A.lv[1].T, A.lv[1].pitch, s1, y1);
        c4 = A.lv[1].children[s1 & ((1 << G::lg(1)) - 1)];
    }
    Stc St;
    stencil(G::uni(0), sp0, w0, St);
    // ---- restriction leg: smoother (:331), get_residual (:338)
    sweeps2(St, rdt, ns, b0[0], b0[1], x0[0], x0[1], p0[0], p0[1]);
    stamp<kMTf>(A, 1);
    if (v0) {
        if constexpr (C > 0)
#pragma unroll
            for (int c = 0; c < 3; ++c) st2(F0 + c * 1024 + 2 * t, make_double2(p0[0][c], p0[1][c]));
#pragma unroll
        for (int k = 0; k < 2; ++k) hs_write(G::uni(0), V0.H, w0, h0[k], p0[k]);
        double r[2][3];
#pragma unroll
        for (int k = 0; k < 2; ++k) residual(St, rdt, p0[k], b0[k], r[k]);
        store3p(V0.RES, V0.pitch, s0, r[0], r[1]);
    }
    stamp<kMTf>(A, 2);
    // ---- prolongation leg (:367-376) from the restriction-leg tnew; with one level,
    //      the 15 coarse smoother calls (:344-359)
    copy3(x0[0], p0[0]);
    copy3(x0[1], p0[1]);
    sweeps2(St, rdt, C > 0 ? ns : ns * A.n_coarse, b0[0], b0[1], x0[0], x0[1], p0[0], p0[1]);
    stamp<kMTf>(A, 3);
    if (v0) {
#pragma unroll
        for (int k = 0; k < 2; ++k) hs_write(G::uni(0), V0.H, w0, h0[k], p0[k]);
        store3p(V0.T, V0.pitch, s0, p0[0], p0[1]);
        store3p(V0.TNN, V0.pitch, s0, x0[0], x0[1]);
    }
    stamp<kMTf>(A, 4);
    // ---- prolongator (:370) on the LDS image (its result is dead, :550)
    if constexpr (C > 0) {
        if (!A.cascade) return;
        __syncthreads();
        if (v1) {
            const int base = (t >> G::lg(1)) << G::lg(0);
            const int fi[4] = {base + c4.x, base + c4.y, base + c4.z, base + c4.w};
            prolong_cascade(F0, 1024, fi, y1);
        }
    }
    stamp<kMTf>(A, 7);
}

template <int S, int L>
hipError_t launch_sl(hipStream_t s, const VArgs &A, unsigned grid, bool coarse) {
    if (coarse) {
        if constexpr (L >= 2)
            hipLaunchKernelGGL((k_vc_coarse<S, L>), dim3(grid), dim3(kMTc), 0, s, A, A.lv[1].stc, A.lv[2].stc,
                               A.lv[3].stc, A.lv[4].stc);
        else
            return hipErrorInvalidValue;
    } else {
        hipLaunchKernelGGL((k_vc_fine<S, L>), dim3(grid), dim3(kMTf), 0, s, A, A.lv[0].stc);
    }
    return hipGetLastError();
}

template <int S>
hipError_t launch_s(hipStream_t s, const VArgs &A, unsigned grid, int L, bool coarse) {
    switch (L) {
        case 1: return launch_sl<S, 1>(s, A, grid, coarse);
        case 2: if constexpr (S >= 2) return launch_sl<S, 2>(s, A, grid, coarse); break;
        case 3: if constexpr (S >= 3) return launch_sl<S, 3>(s, A, grid, coarse); break;
        case 4: if constexpr (S >= 4) return launch_sl<S, 4>(s, A, grid, coarse); break;
        case 5: if constexpr (S >= 5) return launch_sl<S, 5>(s, A, grid, coarse); break;
    }
    return hipErrorInvalidValue;
}

hipError_t launch_part(hipStream_t s, const Level *lv, int L, int U, int n_split, int n_smooth, int n_coarse,
                       double rdt, double *tov, double *tovo, bool coarse) {
    if (!vcycle_fusable(lv, L, n_split, 1, 0, n_smooth)) return hipErrorInvalidValue;
    VArgs A{};
    for (int l = 0; l < L; ++l) {
        const Level &V = lv[l + 1];
        if (V.nsub != (1 << (2 * (n_split - l)))) return hipErrorInvalidValue;
        if ((uint64_t)V.pitch * 3 >= (1ull << 29)) return hipErrorInvalidValue;   // 32-bit byte offsets
        VLevel &o = A.lv[l];
        o.T = V.T; o.TNN = V.TNN; o.RHS = V.RHS; o.RES = V.RES; o.stc = V.stc;
        o.children = (l > 0) ? lv[l].children : nullptr;   // children of level l+1 in level l
        o.pitch = V.pitch;
        const HaloPlan &P = V.halo;
        o.H = HaloArgs{P.d_hsub, P.d_hface, P.d_bcv, P.d_told_halo, tov, tovo, P.d_send, 1 << V.isplit};
    }
    A.U = U;
    A.n_smooth = n_smooth;
    A.n_coarse = n_coarse;
    A.rdt = rdt;
    static const bool diag_nocascade = getenv("PAMG_DIAG_NOCASCADE") != nullptr;
    A.cascade = diag_nocascade ? 0 : 1;
    const int GL = 10 - 2 * n_split;   // 1024 / 4**n_split un_eles per tile
    const unsigned grid = (unsigned)(((int64_t)U + (1 << GL) - 1) >> GL);
    if (grid == 0) return hipSuccess;
    // diagnostics: PAMG_VCYCLE_STAMPS=<file> appends every launch's phase timeline
    static const char *stamp_path = getenv("PAMG_VCYCLE_STAMPS");
    const int waves = (coarse ? kMTc : kMTf) / 64;
    const size_t nst = (size_t)grid * waves * kStampSlots;
    if (stamp_path) {
        hipError_t e = hipMalloc(&A.stamps, nst * sizeof(long long));
        if (e != hipSuccess) return e;
        e = hipMemsetAsync(A.stamps, 0, nst * sizeof(long long), s);
        if (e != hipSuccess) return e;
    }
    hipError_t e = hipErrorInvalidValue;
    switch (n_split) {
        case 1: e = launch_s<1>(s, A, grid, L, coarse); break;
        case 2: e = launch_s<2>(s, A, grid, L, coarse); break;
        case 3: e = launch_s<3>(s, A, grid, L, coarse); break;
        case 4: e = launch_s<4>(s, A, grid, L, coarse); break;
        case 5: e = launch_s<5>(s, A, grid, L, coarse); break;
    }
    if (stamp_path) {
        std::vector<long long> hst(nst);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (e == hipSuccess) e = hipMemcpy(hst.data(), A.stamps, nst * sizeof(long long), hipMemcpyDeviceToHost);
        (void)hipFree(A.stamps);
        if (FILE *f = fopen(stamp_path, "ab")) {
            const long long hdr[4] = {grid, waves, kStampSlots, L * (coarse ? -1 : 1)};
            fwrite(hdr, sizeof hdr, 1, f);
            fwrite(hst.data(), sizeof(long long), nst, f);
            fclose(f);
        }
    }
    return e;
}

}  // namespace

bool vcycle_fusable(const Level *lv, int L, int n_split, int solver, int halo_mode, int n_smooth) {
    (void)lv;
    return solver != 2 && halo_mode == 0 && n_smooth > 0 && L >= 1 && L <= kMaxFusedLevels && n_split <= 5 &&
           n_split >= L;
}

hipError_t launch_vcycle_coarse(hipStream_t s, const Level *lv, int L, int U, int n_split, int n_smooth,
                                int n_coarse, double rdt, double *tov, double *tovo) {
    if (L < 2) return hipSuccess;
    return launch_part(s, lv, L, U, n_split, n_smooth, n_coarse, rdt, tov, tovo, true);
}

hipError_t launch_vcycle_fine(hipStream_t s, const Level *lv, int L, int U, int n_split, int n_smooth,
                              int n_coarse, double rdt, double *tov, double *tovo) {
    return launch_part(s, lv, L, U, n_split, n_smooth, n_coarse, rdt, tov, tovo, false);
}

}  // namespace pamg
