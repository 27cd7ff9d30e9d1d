// Device helpers shared by the kernels of libpamg (gfx950): the per-element
// operator of the reference (get_A_x / get_diagonal / solve_*) and the halo
// words of update_overlaps written by the smoothing threads.
#pragma once

#include <hip/hip_runtime.h>

#include "pamg_internal.h"

namespace pamg {
namespace detail {

constexpr int kBlock = 256;

// The state planes are streamed once per launch (1.2 GB per cycle at n_split = 5, far past the
// 256 MiB Infinity Cache): 16-byte lanes use non-temporal loads and stores (global_load /
// global_store ... nt). Measured on MI355X: the pipelined V-cycle launch 0.244 -> 0.207 ms
// (4.9 -> 6.1 TB/s), the per-step sequence 0.87 -> 0.76 ms per cycle. PAMG_NT is a mask for
// A/B builds: bit 0 non-temporal loads, bit 1 non-temporal stores (0: plain).
#ifndef PAMG_NT
#define PAMG_NT 3
#endif
typedef double v2d_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ double2 ld2(const double *p) {
    if (PAMG_NT & 1) {
        const v2d_t v = __builtin_nontemporal_load(reinterpret_cast<const v2d_t *>(p));
        return make_double2(v.x, v.y);
    }
    return *reinterpret_cast<const double2 *>(p);
}
__device__ __forceinline__ void st2(double *p, double2 v) {
    if (PAMG_NT & 2) {
        const v2d_t w = {v.x, v.y};
        __builtin_nontemporal_store(w, reinterpret_cast<v2d_t *>(p));
        return;
    }
    *reinterpret_cast<double2 *>(p) = v;
}

// The P1 mass matrix of the reference's 3-point edge-midpoint rule is exactly
// M = c [[2,1,1],[1,2,1],[1,1,2]] with c = detwei / 4 (every product N_gi w_g N_gj is
// 0 or 0.25 detwei, detwei equal at the three points of an affine element); the host
// checks this bit for bit (level_stencil). The kernels therefore keep c, not M.
// RN(x / 3) without a division -- the restrictor's mean of three residual components
// (splitting.F90:146-151): q0 = RN(x t) with t = RN(1/3) is within 1 ulp of x / 3, the remainder
// x - 3 q0 is exact in one fma, and one fma correction q0 + r t gives the correctly rounded
// quotient (Markstein's theorem). Outside 2^-1000 <= |x| <= 2^1000 (zeros, subnormals, huge
// values, inf, NaN) it divides. Bitwise x / 3 (scripts/micro/div3_check.c, profiles/r02_div3_check.txt: 2.0e10 values of
// every exponent, 0 differences), in 5 instructions instead of the division's ~10.
#ifndef PAMG_DIV3
#define PAMG_DIV3 1
#endif
__device__ __forceinline__ double div3(double x) {
    if (!PAMG_DIV3) return x / 3.0;   // A/B builds
    const double a = __builtin_fabs(x);
    if (__builtin_expect(!(a >= 0x1p-1000 && a <= 0x1p+1000), 0)) return x / 3.0;
    const double t = 1.0 / 3.0;
    const double q0 = x * t;
    const double r = __builtin_fma(-3.0, q0, x);
    return __builtin_fma(r, t, q0);
}

// The corrected cycle's correction of child q (0..3) of a coarse sub-element with values y (k_interp_add: the
// P1 interpolation the prolongator's cascade encodes, splitting.F90:59-88); the one definition the fused
// forms share, so that each adds the same bits
__device__ __forceinline__ void interp_corr(int q, const double y[3], double add[3]) {
    const double m20 = 0.5 * y[2] + 0.5 * y[0], m12 = 0.5 * y[1] + 0.5 * y[2], m01 = 0.5 * y[0] + 0.5 * y[1];
    switch (q) {
        case 0: add[0] = m20; add[1] = m12; add[2] = y[2]; break;
        case 1: add[0] = m12; add[1] = m20; add[2] = m01; break;
        case 2: add[0] = y[0]; add[1] = m01; add[2] = m20; break;
        default: add[0] = m01; add[1] = y[1]; add[2] = m12; break;
    }
}

struct Stc {
    double c, K[9], w[3];
};

__device__ __forceinline__ void load_stc(const double *__restrict__ rec, Stc &S) {
    S.c = rec[kStcC];
#pragma unroll
    for (int q = 0; q < 9; q += 1) S.K[q] = rec[kStcK + q];
#pragma unroll
    for (int q = 0; q < 3; q += 1) S.w[q] = rec[kStcW + q];
}

// get_A_x (transport_tri_semi.F90:412-448) with theta = 1 and the zero
// advection / flux / surface terms folded: A_i = rdt*(M x)_i + (Kd x)_i.
// (M x)_i is the reference's (M_i1 x_1 + M_i2 x_2) + M_i3 x_3 to the last bit: with
// y_j = c x_j the diagonal product M_ii x_i = (2c) x_i is exactly 2 y_i, so
// M_i1 x_1 + M_i2 x_2 is one fma(2, y_i, y_j) (a single rounding of an exact sum, as
// the reference's add) -- 9 operations instead of 15.
__device__ __forceinline__ void apply_A(const Stc &S, double rdt, const double x[3], double A[3]) {
    const double y0 = S.c * x[0], y1 = S.c * x[1], y2 = S.c * x[2];
    const double mx[3] = {__builtin_fma(2.0, y0, y1) + y2, __builtin_fma(2.0, y1, y0) + y2,
                          __builtin_fma(2.0, y2, y0 + y1)};
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        double kx = S.K[3 * i] * x[0] + S.K[3 * i + 1] * x[1] + S.K[3 * i + 2] * x[2];
        A[i] = rdt * mx[i] + kx;
    }
}

// One sweep of solve_Gauss_Seidel / solve_Jacobi (:491-507), which coincide
// for the block-diagonal operator: x_i += (omega / D_i) * (b_i - A_i).
__device__ __forceinline__ void sweep(const Stc &S, double rdt, const double b[3], double x[3]) {
    double A[3];
    apply_A(S, rdt, x, A);
#pragma unroll
    for (int i = 0; i < 3; ++i) x[i] = x[i] + S.w[i] * (b[i] - A[i]);
}

// get_residual's residuale = A x - RHS (:869), reference order
__device__ __forceinline__ void resid(const Stc &S, double rdt, const double x[3], const double b[3], double r[3]) {
    double A[3];
    apply_A(S, rdt, x, A);
#pragma unroll
    for (int i = 0; i < 3; ++i) r[i] = A[i] - b[i];
}

// Contracted operator (pamg_params.arith = 1): the element matrix A = (1/dt) M + Kd is
// assembled once per un_ele on the host (operator record, kStcA) and every row is one
// fma chain -- a sweep is 12 fp64 operations with a dependence depth of 4 (39 and 8 in
// the reference's order). Same algebra as get_A_x / solve_Jacobi (:412-497); the
// roundings differ (within 1e-13 relative of the reference, tests/test_gpu_parity.py).
struct StcF {
    double A[9], w[3];
};

__device__ __forceinline__ void load_stc(const double *__restrict__ rec, StcF &S) {
#pragma unroll
    for (int q = 0; q < 9; q += 1) S.A[q] = rec[kStcA + q];
#pragma unroll
    for (int q = 0; q < 3; q += 1) S.w[q] = rec[kStcW + q];
}

// x_i += w_i (b_i - sum_j A_ij x_j), all rows from the old x (Jacobi = Gauss-Seidel here)
__device__ __forceinline__ void sweep(const StcF &S, double, const double b[3], double x[3]) {
    double t[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        t[i] = __builtin_fma(-S.A[3 * i], x[0], b[i]);
        t[i] = __builtin_fma(-S.A[3 * i + 1], x[1], t[i]);
        t[i] = __builtin_fma(-S.A[3 * i + 2], x[2], t[i]);
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) x[i] = __builtin_fma(S.w[i], t[i], x[i]);
}

__device__ __forceinline__ void resid(const StcF &S, double, const double x[3], const double b[3], double r[3]) {
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        double t = __builtin_fma(S.A[3 * i], x[0], -b[i]);
        t = __builtin_fma(S.A[3 * i + 1], x[1], t);
        r[i] = __builtin_fma(S.A[3 * i + 2], x[2], t);
    }
}

// solve_Richardson (:511-518, solver = 2): the smoother zeroes its mass, stiffness and flux terms
// (:585-612), so a sweep is x_i + omega (b_i - (0 - 0 + 0)) = x_i + omega b_i, the reference's two
// roundings (no contraction); get_residual keeps the full operator in the reference's order (the
// contracted arithmetic is for solvers 1 and 3, pamg_params.arith)
struct StcR {
    Stc s;
    double om;
};

__device__ __forceinline__ void load_stc(const double *__restrict__ rec, StcR &S) {
    load_stc(rec, S.s);
    S.om = rec[kStcOm];
}

__device__ __forceinline__ void sweep(const StcR &S, double, const double b[3], double x[3]) {
#pragma unroll
    for (int i = 0; i < 3; ++i) x[i] = x[i] + S.om * b[i];
}

__device__ __forceinline__ void resid(const StcR &S, double rdt, const double x[3], const double b[3], double r[3]) {
    resid(S.s, rdt, x, b, r);
}

// Halo words written by the smoother (update_overlaps, splitting.F90:1210-1397).
struct HaloArgs {
    const int4 *hsub;     // per sub-element: position along faces 1, 2, 3 (0 = none)
    const int4 *hface;    // per (un_ele, face): {mode | rev << 2, dst base, aux, 0}
    const double2 *bcv;   // boundary values sin(x + y) at the two face nodes
    const double *told;   // told values of the copied sub-elements (3 per entry, hface.w = first entry)
    double *tov, *tovo, *send;
    int m;                // 2**i_split sub-elements per face
};

// Words another workgroup of the same launch reads (the persistent face-operator chain,
// pamg_face.hip k_face_chain): written through to the device-coherent level (a relaxed agent-scope
// atomic store of the 8-byte pattern on a global-address-space pointer: global_store_dwordx2 sc1)
// and read the same way (global_load_dwordx2 sc1, which bypasses this CU's L1), the hand-off form
// of cdna_hip_programming.md 6 Guideline 16 (R1) with one workgroup per CU
typedef __attribute__((address_space(1))) unsigned long long g_u64;
typedef __attribute__((address_space(1))) unsigned g_u32;
__device__ __forceinline__ void st_coh(double *p, double x) {
    __hip_atomic_store((g_u64 *)p, (unsigned long long)__double_as_longlong(x), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_coh(const double *p) {
    return __longlong_as_double(
        (long long)__hip_atomic_load((g_u64 *)const_cast<double *>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
template <bool COH>
__device__ __forceinline__ void st_halo(double *p, double x) {
    if constexpr (COH) st_coh(p, x);
    else *p = x;
}

// The reference rewrites the halo at the start of every sweep from the then
// current tnew (:550-556); the last write of a smoother call therefore carries
// the iterate before the last sweep, which is what these threads hold in p[].
// The halo metadata (face positions, face records, told) is fetched before the
// sweeps so its latency hides under the arithmetic.
// TNEW / STATIC select the words written: TNEW the tnew copies (t_overlap of a
// neighbour on this rank, the tnew half of a send entry); STATIC the words that do
// not change within a time step (t_overlap_old from told, the boundary values of
// both arrays, the told half of a send entry). The per-step kernels write both;
// the fused V-cycle writes TNEW only and leaves STATIC to k_overlap_static.
// COH: the t_overlap words are written through (st_coh) for readers in other workgroups
// SCOH: the tnew half of a send entry is written through (the resident call's early exchange reads
// the send buffer while the launch still runs, pamg_api.cpp vcycle_fused)
template <bool TNEW = true, bool STATIC = true, bool COH = false, bool SCOH = false>
__device__ __forceinline__ void halo_face(const HaloArgs &H, int4 rec, int f, int i, const double t[3],
                                          const double to[3]) {
    const int mode = rec.x & 3;
    if (mode == 0) {   // domain boundary: BC values into the own column (:1243-1252, :1287-1295, :1345-1353)
        if (!STATIC) return;
        const int a = (i - 1) * 3 + (f == 3 ? 1 : 0);
        const int b = (i - 1) * 3 + (f == 2 ? 1 : 2);
        const double2 v = H.bcv[rec.z + i - 1];
        st_halo<COH>(H.tov + rec.y + a, v.x);
        st_halo<COH>(H.tov + rec.y + b, v.y);
        H.tovo[rec.y + a] = v.x;
        H.tovo[rec.y + b] = v.y;
    } else if (mode == 1) {   // neighbour on this rank: t_overlap(slot, Nside) of the neighbour
        const int k = (rec.x >> 2) ? (H.m - i + 1) : i;
        const int64_t d = rec.y + (int64_t)(k - 1) * 3;
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            if (TNEW) st_halo<COH>(H.tov + d + c, t[c]);
            if (STATIC) H.tovo[d + c] = to[c];
        }
    } else {                  // neighbour on another rank: packed send buffer (RCCL)
        double *o = H.send + 6 * (int64_t)(rec.z + i - 1);
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            if (TNEW) st_halo<SCOH>(o + c, t[c]);
            if (STATIC) o[3 + c] = to[c];
        }
    }
}

struct HaloPre {
    int4 hs0, hs1;              // face positions of the two sub-elements
    int4 r1, r2, r3;            // face records (faces 1, 2, 3) of the un_ele
    double a0, a1, a2, c0, c1, c2;   // told of the two sub-elements (compact told halo)
    bool any;
};

// entry of the compact told halo holding a boundary sub-element's told (-1: none)
__device__ __forceinline__ int told_entry(const HaloPre &P, int4 hs) {
    if (hs.x && (P.r1.x & 3)) return P.r1.w + hs.x - 1;
    if (hs.y && (P.r2.x & 3)) return P.r2.w + hs.y - 1;
    if (hs.z && (P.r3.x & 3)) return P.r3.w + hs.z - 1;
    return -1;
}

__device__ __forceinline__ void halo_prefetch(const HaloArgs &H, int64_t s, int64_t u, int nsub_log2, HaloPre &P) {
    const int64_t sub = s & ((1ll << nsub_log2) - 1);
    P.hs0 = H.hsub[sub];
    P.hs1 = H.hsub[sub + 1];
    P.any = (P.hs0.x | P.hs0.y | P.hs0.z | P.hs1.x | P.hs1.y | P.hs1.z) != 0;
    P.a0 = P.a1 = P.a2 = P.c0 = P.c1 = P.c2 = 0.0;
    if (P.any) {
        P.r1 = H.hface[3 * u];
        P.r2 = H.hface[3 * u + 1];
        P.r3 = H.hface[3 * u + 2];
        const int e0 = told_entry(P, P.hs0), e1 = told_entry(P, P.hs1);
        if (e0 >= 0) { P.a0 = H.told[3 * (int64_t)e0]; P.a1 = H.told[3 * (int64_t)e0 + 1]; P.a2 = H.told[3 * (int64_t)e0 + 2]; }
        if (e1 >= 0) { P.c0 = H.told[3 * (int64_t)e1]; P.c1 = H.told[3 * (int64_t)e1 + 1]; P.c2 = H.told[3 * (int64_t)e1 + 2]; }
    }
}

template <bool COH = false>
__device__ __forceinline__ void halo_write(const HaloArgs &H, const HaloPre &P, const double p0[3],
                                           const double p1[3]) {
    if (!P.any) return;
    const double t0[3] = {P.a0, P.a1, P.a2}, t1[3] = {P.c0, P.c1, P.c2};
    if (P.hs0.x) halo_face<true, true, COH>(H, P.r1, 1, P.hs0.x, p0, t0);
    if (P.hs0.y) halo_face<true, true, COH>(H, P.r2, 2, P.hs0.y, p0, t0);
    if (P.hs0.z) halo_face<true, true, COH>(H, P.r3, 3, P.hs0.z, p0, t0);
    if (P.hs1.x) halo_face<true, true, COH>(H, P.r1, 1, P.hs1.x, p1, t1);
    if (P.hs1.y) halo_face<true, true, COH>(H, P.r2, 2, P.hs1.y, p1, t1);
    if (P.hs1.z) halo_face<true, true, COH>(H, P.r3, 3, P.hs1.z, p1, t1);
}


// The cascaded source term s' of one level-1 sub-element (get_RHS :452-464 with the source
// term :593): s_j = -2k sin(x_j + y_j) at the get_splitting node coordinates, cascaded in place
// through M (s'_1 = (M s)_1, s'_2 = M_21 s'_1 + M_22 s_2 + M_23 s_3, ...), the reference's
// operation order. It depends on the geometry only: k_source forms it once at upload.
__device__ __forceinline__ void source_one(const double *__restrict__ g, const double *__restrict__ M, int2 ri,
                                           double k, double src[3]) {
    const int irow = ri.x, ipos = ri.y;
    double xl[3][2];
#pragma unroll
    for (int d = 0; d < 2; ++d) {
        const double x3 = g[d], v1 = g[2 + d], v2 = g[4 + d];
        if (ipos % 2 != 0) {
            xl[2][d] = x3 + (double)(irow - 1) * v2 + (double)(ipos / 2) * v1;
            xl[1][d] = x3 + (double)irow * v2 + (double)(ipos / 2) * v1;
            xl[0][d] = x3 + (double)(irow - 1) * v2 + v1 * (double)(ipos / 2 + 1);
        } else {
            xl[0][d] = x3 + (double)irow * v2 + v1 * (double)(ipos / 2 - 1);
            xl[1][d] = x3 + (double)(irow - 1) * v2 + v1 * (double)(ipos / 2);
            xl[2][d] = x3 + (double)irow * v2 + v1 * (double)(ipos / 2);
        }
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) src[i] = -(2 * k * sin(xl[i][0] + xl[i][1]));
#pragma unroll
    for (int i = 0; i < 3; ++i) src[i] = M[3 * i] * src[0] + M[3 * i + 1] * src[1] + M[3 * i + 2] * src[2];
}

// Level-1 RHS of one sub-element from its told t and its s' (get_RHS :452-464):
// RHS_i = rdt (M t)_i + s'_i, the reference's operation order; (M t)_i is evaluated from
// c = M_12 as in apply_A, bit for bit the reference's (M_i1 t_1 + M_i2 t_2) + M_i3 t_3.
// Shared by k_rhs and the pipelined V-cycle launch that starts a time step (RHSF).
__device__ __forceinline__ void rhs_from_source(double c, double rdt, const double t[3], const double src[3],
                                                double rhs[3]) {
    const double y0 = c * t[0], y1 = c * t[1], y2 = c * t[2];
    const double mx[3] = {__builtin_fma(2.0, y0, y1) + y2, __builtin_fma(2.0, y1, y0) + y2,
                          __builtin_fma(2.0, y2, y0 + y1)};
#pragma unroll
    for (int i = 0; i < 3; ++i) rhs[i] = rdt * mx[i] + src[i];
}

}  // namespace detail
}  // namespace pamg
