// HIP kernels of the multigrid hot path, written for CDNA4 (gfx950).
//
// Data layout in HBM: every level field is three fp64 planes [3][pitch]
// (structure of arrays, sub-element index s = u * nsub + str_ele - 1), so a
// wave64 moves 1 KiB per plane per instruction with 16-B (double2) lanes.
// Each thread owns two consecutive sub-elements, which always belong to the
// same un_ele (nsub = 4**i_split >= 4), so the 256-B operator record of that
// un_ele is read once per thread and served from L1/L2 to all lanes of the
// un_ele. The arithmetic is the reference's, in its order and without FMA
// contraction (built with -ffp-contract=off): results are bit-identical to
// the reference's fp64 build except where the device sine enters (level-1
// source term).
//
// The operator is block diagonal (3x3 per sub-element): the
// work per sub-element per sweep is ~30 flop on 72-168 B, far left of the
// fp64 ridge, so these are HBM-bound streaming kernels; MFMA has no role.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>

#include "pamg_device.h"
#include "pamg_internal.h"

namespace pamg {
namespace {

using namespace detail;

// Gather of told at the halo's copied sub-elements (entry order (u, f, i)),
// run when told changes (time-step start, set_state), not per smoother call.
__global__ __launch_bounds__(kBlock) void k_told_halo(const double *__restrict__ TOLD, int64_t pitch,
                                                      const int4 *__restrict__ hface, const int *__restrict__ surf,
                                                      double *__restrict__ out, int U, int m, int nsub_log2) {
    const int64_t idx = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (idx >= (int64_t)U * 3 * m) return;
    const int i = (int)(idx % m) + 1;
    const int f = (int)((idx / m) % 3) + 1;
    const int64_t q = idx / (3 * m);
    const int4 rec = hface[3 * q + f - 1];
    if ((rec.x & 3) == 0) return;
    const int64_t s = (q << nsub_log2) + surf[(i - 1) + (f - 1) * m] - 1;
    double *o = out + 3 * (int64_t)(rec.w + i - 1);
#pragma unroll
    for (int c = 0; c < 3; ++c) o[c] = TOLD[c * pitch + s];
}

// The halo words that are constant within a time step (t_overlap_old from told, the
// boundary values sin(x + y) of both arrays, the told half of the send entries), as
// the level's smoother writes them (update_overlaps, splitting.F90:1210-1397); one
// thread per (un_ele, face, position), the order of k_told_halo. The fused V-cycle
// writes only the tnew words; this kernel runs before its first launch in a time step.
// TOLD != null (pamg_run's steps): told straight from the TOLD planes, and the compact told copy
// of k_told_halo written on the way (same threads, same words: one launch instead of two).
__global__ __launch_bounds__(kBlock) void k_overlap_static(HaloArgs H, const int *__restrict__ surf, int U,
                                                           const double *__restrict__ TOLD, int64_t pitch,
                                                           int nsub_log2) {
    const int m = H.m;
    const int64_t idx = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (idx >= (int64_t)U * 3 * m) return;
    const int i = (int)(idx % m) + 1;
    const int f = (int)((idx / m) % 3) + 1;
    const int64_t q = idx / (3 * m);
    const int4 rec = H.hface[3 * q + f - 1];
    double to[3] = {0.0, 0.0, 0.0};
    if (TOLD) {
        if (rec.x & 3) {
            const int64_t s = (q << nsub_log2) + surf[(i - 1) + (f - 1) * m] - 1;
            double *o = const_cast<double *>(H.told) + 3 * (int64_t)(rec.w + i - 1);   // d_told_halo
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                to[c] = TOLD[c * pitch + s];
                o[c] = to[c];
            }
        }
    } else if (rec.x & 3) {
        // the sub-element's told sits in the compact told halo at its first copied face
        const int sub = surf[(i - 1) + (f - 1) * m] - 1;
        const int4 hs = H.hsub[sub];
        const int4 r[3] = {H.hface[3 * q], H.hface[3 * q + 1], H.hface[3 * q + 2]};
        const int pos[3] = {hs.x, hs.y, hs.z};
        int e = -1;
        for (int g = 0; g < 3 && e < 0; ++g)
            if (pos[g] && (r[g].x & 3)) e = r[g].w + pos[g] - 1;
        if (e >= 0)
#pragma unroll
            for (int c = 0; c < 3; ++c) to[c] = H.told[3 * (int64_t)e + c];
    }
    halo_face<false, true>(H, rec, f, i, to, to);
}

// Fused smoother call(s): `sweeps` consecutive sweeps kept in registers.
// Reference semantics (:548-550): each sweep starts with tnew := tnew_nonlin,
// so after the call tnew holds the iterate before the last sweep and
// tnew_nonlin the last one. `src` may alias T or TNN (each thread reads its
// own words before writing them). UNIFORM: every wave lies inside one un_ele
// (nsub >= 128), so the operator record is read through the scalar unit.
template <bool RICHARDSON, bool UNIFORM, class ST = Stc>
__global__ __launch_bounds__(kBlock) void k_smooth(const double *src, double *T, double *TNN,
                                                   const double *__restrict__ RHS,
                                                   const double *__restrict__ stc, int64_t pitch,
                                                   int64_t npairs, int nsub_log2, int sweeps, double rdt,
                                                   double omega, HaloArgs H) {
    const int64_t p = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (p >= npairs) return;
    const int64_t s = 2 * p;
    int64_t u = s >> nsub_log2;
    if (UNIFORM) u = __builtin_amdgcn_readfirstlane((int)u);
    double2 xv[3], bv[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        xv[c] = ld2(src + c * pitch + s);
        bv[c] = ld2(RHS + c * pitch + s);
    }
    HaloPre hp;
    hp.any = false;
    if (H.hsub) halo_prefetch(H, s, u, nsub_log2, hp);
    double x0[3] = {xv[0].x, xv[1].x, xv[2].x}, x1[3] = {xv[0].y, xv[1].y, xv[2].y};
    const double b0[3] = {bv[0].x, bv[1].x, bv[2].x}, b1[3] = {bv[0].y, bv[1].y, bv[2].y};
    double p0[3] = {x0[0], x0[1], x0[2]}, p1[3] = {x1[0], x1[1], x1[2]};
    if (RICHARDSON) {
        // solve_Richardson (:511-518): mass/stiff/flux terms are reset to 0 (:585-612)
        for (int it = 0; it < sweeps; ++it) {
#pragma unroll
            for (int i = 0; i < 3; ++i) {
                p0[i] = x0[i]; p1[i] = x1[i];
                x0[i] = x0[i] + omega * (b0[i] - (0.0 - 0.0 + 0.0));
                x1[i] = x1[i] + omega * (b1[i] - (0.0 - 0.0 + 0.0));
            }
        }
    } else {
        ST S;
        load_stc(stc + u * kStcStride, S);
        for (int it = 0; it < sweeps; ++it) {
#pragma unroll
            for (int i = 0; i < 3; ++i) { p0[i] = x0[i]; p1[i] = x1[i]; }
            sweep(S, rdt, b0, x0);
            sweep(S, rdt, b1, x1);
        }
    }
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        st2(T + c * pitch + s, make_double2(p0[c], p1[c]));
        st2(TNN + c * pitch + s, make_double2(x0[c], x1[c]));
    }
    halo_write(H, hp, p0, p1);
}

// get_residual (:725-873): residuale = A x - RHS (note the sign, :869); NEG: RHS - A x (the
// corrected cycle's residual, pamg_params.cycle = 1)
template <class ST, bool NEG = false>
__global__ __launch_bounds__(kBlock) void k_residual(const double *__restrict__ T, const double *__restrict__ RHS,
                                                     double *__restrict__ RES, const double *__restrict__ stc,
                                                     int64_t pitch, int64_t npairs, int nsub_log2, double rdt) {
    const int64_t p = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (p >= npairs) return;
    const int64_t s = 2 * p;
    double2 xv[3], bv[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        xv[c] = ld2(T + c * pitch + s);
        bv[c] = ld2(RHS + c * pitch + s);
    }
    ST S;
    load_stc(stc + (s >> nsub_log2) * kStcStride, S);
    const double x0[3] = {xv[0].x, xv[1].x, xv[2].x}, x1[3] = {xv[0].y, xv[1].y, xv[2].y};
    const double b0[3] = {bv[0].x, bv[1].x, bv[2].x}, b1[3] = {bv[0].y, bv[1].y, bv[2].y};
    double r0[3], r1[3];
    resid(S, rdt, x0, b0, r0);
    resid(S, rdt, x1, b1, r1);
#pragma unroll
    for (int c = 0; c < 3; ++c) st2(RES + c * pitch + s, NEG ? make_double2(-r0[c], -r1[c]) : make_double2(r0[c], r1[c]));
}

// corrected cycle: tnew_l += P tnew_{l+1}, the P1 interpolation the prolongator's cascade
// (splitting.F90:59-88) encodes, applied to the coarse correction alone; one thread per
// coarse sub-element (its four children are its own: fine 4c .. 4c+3 in the storage order)
// one thread per FINE sub-element f (child q = f & 3 of coarse c = f >> 2, Level::pos): coalesced
// read-modify-writes of the fine planes (a thread per coarse sub-element touching its four
// children made 8-byte accesses 32 bytes apart and ran at ~0.2 TB/s); the coarse values are read
// by the four consecutive threads of its children
__global__ __launch_bounds__(kBlock) void k_interp_add(double *T, const double *__restrict__ Tc, int64_t pitch_f,
                                                       int64_t pitch_c, int64_t Nc) {
    const int64_t f = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (f >= 4 * Nc) return;
    const int64_t c = f >> 2;
    const int q = (int)(f & 3);
    const double y[3] = {Tc[c], Tc[pitch_c + c], Tc[2 * pitch_c + c]};
    double add[3];
    interp_corr(q, y, add);   // the P1 interpolation of the prolongator cascade (splitting.F90:59-88)
#pragma unroll
    for (int i = 0; i < 3; ++i) T[i * pitch_f + f] = T[i * pitch_f + f] + add[i];
}

// Level-1 right-hand side + time-step start (:316-317, :593, get_RHS :452-464):
// told := tnew, tnew_nonlin := tnew, RHS_i = rdt (M told)_i + s'_i with the cascaded source
// term s' precomputed by k_source (the reference recomputes it, with three sines per node, at
// every visit; it depends on the geometry only). start_of_step 2: the same without the
// tnew_nonlin store (pamg_run: the V-cycle that follows rewrites it before any read, :327).
// One adjacent pair of sub-elements per thread (same un_ele: nsub is a power of 4), the
// state planes streamed with 16-byte non-temporal accesses (ld2 / st2). told_halo (start of a
// step): also the compact told copy of k_told_halo, from the told values in registers.
__global__ __launch_bounds__(kBlock) void k_rhs(const double *__restrict__ T, double *TOLD,
                                                double *__restrict__ TNN, double *__restrict__ RHS,
                                                const double *__restrict__ SRC, const double *__restrict__ stc,
                                                int64_t pitch, int64_t N, int nsub_log2, double rdt,
                                                int start_of_step, const int4 *__restrict__ hsub,
                                                const int4 *__restrict__ hface, double *__restrict__ told_halo) {
    const int64_t s = 2 * ((int64_t)blockIdx.x * kBlock + threadIdx.x);
    if (s >= N) return;
    const int64_t u = s >> nsub_log2;
    const int sub = (int)(s & ((1ll << nsub_log2) - 1));
    double t0[3], t1[3], q0[3], q1[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        const double2 v = ld2((start_of_step ? T : TOLD) + c * pitch + s);
        const double2 w = ld2(SRC + c * pitch + s);
        t0[c] = v.x;
        t1[c] = v.y;
        q0[c] = w.x;
        q1[c] = w.y;
        if (start_of_step) {
            st2(TOLD + c * pitch + s, v);
            if (start_of_step == 1) st2(TNN + c * pitch + s, v);
        }
    }
    if (told_halo) {   // the compact told copy of the halo's sub-elements (k_told_halo's words)
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const int4 hs = hsub[sub + q];
            const int pos[3] = {hs.x, hs.y, hs.z};
#pragma unroll
            for (int f = 0; f < 3; ++f) {
                if (!pos[f]) continue;
                const int4 rec = hface[3 * u + f];
                if ((rec.x & 3) == 0) continue;
                double *o = told_halo + 3 * (int64_t)(rec.w + pos[f] - 1);
#pragma unroll
                for (int c = 0; c < 3; ++c) o[c] = q ? t1[c] : t0[c];
            }
        }
    }
    const double c = stc[u * kStcStride + kStcC];
    double r0[3], r1[3];
    rhs_from_source(c, rdt, t0, q0, r0);
    rhs_from_source(c, rdt, t1, q1, r1);
#pragma unroll
    for (int c = 0; c < 3; ++c) st2(RHS + c * pitch + s, make_double2(r0[c], r1[c]));
}

// The cascaded source term s' of every level-1 sub-element (source_one), once at upload.
__global__ __launch_bounds__(kBlock) void k_source(double *__restrict__ SRC, const double *__restrict__ stc,
                                                   const double *__restrict__ geo, const int2 *__restrict__ subinfo,
                                                   int64_t pitch, int64_t N, int nsub_log2, double k) {
    const int64_t s = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (s >= N) return;
    const int64_t u = s >> nsub_log2;
    const int sub = (int)(s & ((1ll << nsub_log2) - 1));
    double q[3];
    source_one(geo + u * kGeoStride, stc + u * kStcStride + kStcM, subinfo[sub], k, q);
#pragma unroll
    for (int c = 0; c < 3; ++c) SRC[c * pitch + s] = q[c];
}

// LDS-tiled inter-level transfers. A workgroup owns an aligned tile of TF fine
// sub-elements, which carries its own TF / 4 coarse sub-elements (the storage order puts the
// children of coarse g at fine 4g .. 4g+3, pamg_internal.h Level::pos): the fine fields of
// the tile are streamed into LDS with coalesced double2 loads, the children of each coarse
// sub-element (element_conversion, splitting.F90:97-140) are addressed in LDS at tile-local
// 4cc .. 4cc+3, and the tile is streamed back.
__global__ __launch_bounds__(kBlock) void k_prolong_tile(double *T, double *TNN, const double *__restrict__ Tc,
                                                         int64_t pitch_f, int64_t pitch_c, int64_t Nf, int tile_log2,
                                                         int write_tnn) {
    extern __shared__ __attribute__((aligned(16))) double lds[];
    const int TF = 1 << tile_log2;
    const int64_t f0 = (int64_t)blockIdx.x << tile_log2;
    const int nf = (int)min((int64_t)TF, Nf - f0);
    for (int j = 2 * threadIdx.x; j < nf; j += 2 * kBlock) {
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            const double2 v = ld2(T + c * pitch_f + f0 + j);
            *reinterpret_cast<double2 *>(&lds[c * TF + j]) = v;
            if (write_tnn) st2(TNN + c * pitch_f + f0 + j, v);   // tnew_nonlin := tnew (:365-367)
        }
    }
    __syncthreads();
    const int64_t c0 = f0 >> 2;
    for (int cc = threadIdx.x; cc < (nf >> 2); cc += kBlock) {
        const int fi[4] = {4 * cc, 4 * cc + 1, 4 * cc + 2, 4 * cc + 3};
        const double y[3] = {Tc[c0 + cc], Tc[pitch_c + c0 + cc], Tc[2 * pitch_c + c0 + cc]};
        double f[4][3];
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int i = 0; i < 3; ++i) f[q][i] = lds[i * TF + fi[q]];
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
            for (int i = 0; i < 3; ++i) lds[i * TF + fi[q]] = f[q][i];
    }
    __syncthreads();
    for (int j = 2 * threadIdx.x; j < nf; j += 2 * kBlock)
#pragma unroll
        for (int c = 0; c < 3; ++c) st2(T + c * pitch_f + f0 + j, *reinterpret_cast<const double2 *>(&lds[c * TF + j]));
}

__global__ __launch_bounds__(kBlock) void k_restrict_tile(const double *__restrict__ RES, double *__restrict__ RHSc,
                                                          int64_t pitch_f, int64_t pitch_c, int64_t Nf, int tile_log2) {
    extern __shared__ __attribute__((aligned(16))) double lds[];
    const int TF = 1 << tile_log2;
    const int64_t f0 = (int64_t)blockIdx.x << tile_log2;
    const int nf = (int)min((int64_t)TF, Nf - f0);
    for (int j = 2 * threadIdx.x; j < nf; j += 2 * kBlock)
#pragma unroll
        for (int c = 0; c < 3; ++c)
            *reinterpret_cast<double2 *>(&lds[c * TF + j]) = ld2(RES + c * pitch_f + f0 + j);
    __syncthreads();
    const int64_t c0 = f0 >> 2;
    for (int cc = threadIdx.x; cc < (nf >> 2); cc += kBlock) {
        const int pick[3] = {4 * cc + 2, 4 * cc + 3, 4 * cc};   // children 3, 4, 1 (splitting.F90:26-28)
#pragma unroll
        for (int i = 0; i < 3; ++i)
            RHSc[i * pitch_c + c0 + cc] = div3(lds[pick[i]] + lds[TF + pick[i]] + lds[2 * TF + pick[i]]);
    }
}

// restrictor(l) followed by get_residual(l) (:336, :338) in one pass over an
// aligned tile of fine sub-elements: the previous cycle's residual is staged in LDS and
// restricted into RHS_{l+1}; then the new residual A tnew - RHS overwrites it.
// ITER = tile / 512: every thread issues all its loads (old residual, tnew,
// RHS) before the tile barrier, so the three streams are in flight together.
template <bool UNIFORM, int ITER, class ST = Stc>
__global__ __launch_bounds__(kBlock) void k_restrict_residual(const double *__restrict__ T,
                                                              const double *__restrict__ RHS, double *RES,
                                                              double *__restrict__ RHSc,
                                                              const double *__restrict__ stc, int64_t pitch_f,
                                                              int64_t pitch_c, int64_t Nf, int nsubf_log2, double rdt) {
    extern __shared__ __attribute__((aligned(16))) double lds[];
    constexpr int TF = ITER * 2 * kBlock;
    const int64_t f0 = (int64_t)blockIdx.x * TF;
    const int nf = (int)min((int64_t)TF, Nf - f0);
    double2 r[ITER][3], x[ITER][3], b[ITER][3];
#pragma unroll
    for (int it = 0; it < ITER; ++it) {
        const int j = 2 * threadIdx.x + it * 2 * kBlock;
        if (j < nf) {
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                r[it][c] = ld2(RES + c * pitch_f + f0 + j);
                x[it][c] = ld2(T + c * pitch_f + f0 + j);
                b[it][c] = ld2(RHS + c * pitch_f + f0 + j);
            }
        }
    }
#pragma unroll
    for (int it = 0; it < ITER; ++it) {
        const int j = 2 * threadIdx.x + it * 2 * kBlock;
        if (j < nf) {
#pragma unroll
            for (int c = 0; c < 3; ++c) *reinterpret_cast<double2 *>(&lds[c * TF + j]) = r[it][c];
        }
    }
    __syncthreads();
    const int64_t c0 = f0 >> 2;
    for (int cc = threadIdx.x; cc < (nf >> 2); cc += kBlock) {
        const int pick[3] = {4 * cc + 2, 4 * cc + 3, 4 * cc};
#pragma unroll
        for (int i = 0; i < 3; ++i)
            RHSc[i * pitch_c + c0 + cc] = div3(lds[pick[i]] + lds[TF + pick[i]] + lds[2 * TF + pick[i]]);
    }
#pragma unroll
    for (int it = 0; it < ITER; ++it) {
        const int j = 2 * threadIdx.x + it * 2 * kBlock;
        if (j >= nf) continue;
        const int64_t s = f0 + j;
        int64_t u = s >> nsubf_log2;
        if (UNIFORM) u = __builtin_amdgcn_readfirstlane((int)u);
        ST S;
        load_stc(stc + u * kStcStride, S);
        const double x0[3] = {x[it][0].x, x[it][1].x, x[it][2].x}, x1[3] = {x[it][0].y, x[it][1].y, x[it][2].y};
        const double b0[3] = {b[it][0].x, b[it][1].x, b[it][2].x}, b1[3] = {b[it][0].y, b[it][1].y, b[it][2].y};
        double r0[3], r1[3];
        resid(S, rdt, x0, b0, r0);
        resid(S, rdt, x1, b1, r1);
#pragma unroll
        for (int c = 0; c < 3; ++c) st2(RES + c * pitch_f + s, make_double2(r0[c], r1[c]));
    }
}

// Unpack of the halo words received from other ranks (RCCL) into t_overlap.
__global__ __launch_bounds__(kBlock) void k_halo_unpack(const double *__restrict__ recv, const int *__restrict__ dst,
                                                        int n, double *__restrict__ tov, double *__restrict__ tovo) {
    const int e = blockIdx.x * kBlock + threadIdx.x;
    if (e >= n) return;
    const int d = dst[e];
#pragma unroll
    for (int q = 0; q < 3; ++q) {
        tov[d + q] = recv[6 * (int64_t)e + q];
        tovo[d + q] = recv[6 * (int64_t)e + 3 + q];
    }
}

__global__ __launch_bounds__(kBlock) void k_halo_unpack3(const double *__restrict__ recv, const int *__restrict__ dst,
                                                         int n, double *__restrict__ tov) {
    const int e = blockIdx.x * kBlock + threadIdx.x;
    if (e >= n) return;
    const int d = dst[e];
#pragma unroll
    for (int q = 0; q < 3; ++q) tov[d + q] = recv[3 * (int64_t)e + q];
}

// device-to-device copy of whole planes (tnew_nonlin := tnew, told := tnew)
__global__ __launch_bounds__(kBlock) void k_copy(const double *__restrict__ a, double *__restrict__ b, int64_t n2) {
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n2; i += (int64_t)gridDim.x * kBlock)
        st2(b + 2 * i, ld2(a + 2 * i));
}

// layout converters between the reference's (3, nsub, U) -- str_ele in its row-wise
// numbering -- and the planes in the storage order (pos[e]: position of str_ele e + 1)
__global__ __launch_bounds__(kBlock) void k_to_soa(const double *__restrict__ aos, double *__restrict__ soa,
                                                   const int *__restrict__ pos, int64_t N, int64_t pitch,
                                                   int nsub_log2) {
    const int64_t s = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (s >= N) return;
    const int64_t d = ((s >> nsub_log2) << nsub_log2) + pos[s & ((1ll << nsub_log2) - 1)];
#pragma unroll
    for (int c = 0; c < 3; ++c) soa[c * pitch + d] = aos[3 * s + c];
}
__global__ __launch_bounds__(kBlock) void k_to_aos(const double *__restrict__ soa, double *__restrict__ aos,
                                                   const int *__restrict__ pos, int64_t N, int64_t pitch,
                                                   int nsub_log2) {
    const int64_t s = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (s >= N) return;
    const int64_t d = ((s >> nsub_log2) << nsub_log2) + pos[s & ((1ll << nsub_log2) - 1)];
#pragma unroll
    for (int c = 0; c < 3; ++c) aos[3 * s + c] = soa[c * pitch + d];
}

// ---- roofline kernels: one unfused level-1 sweep -------------------------
// Assembled operator (the north star's "element-block-sparse" matrix in the
// block-CSR layout of matrices.F90:997-1198 with its single non-zero block per
// block-row): per sub-element the 3x3 block A_e = (1/dt) M + Kd (9 planes, the
// operator record's kStcA words, assembled on the host in fp64) and w = omega/D
// (3 planes). Traffic per sub-element: x 24 + b 24 + out 24 + A 72 + w 24 = 168 B
// (SURVEY.md 8d). The sweep is the contracted arithmetic of arith = 1 (one fma chain
// per row, pamg_device.h StcF): bitwise the oracle's orc_sweep_once(arith = 1).
// Layout of the assembled blocks (round 5's A/B, kAsmLayout below):
//   0  twelve SoA planes (blk[q pitch + s]): 18 load streams + 3 store streams a launch, the planes N
//      doubles (64 MiB at n_split = 5) apart -- 0.63-0.69 of 8 TB/s across boxes (round 4);
//   1  tiled: per tile of kAsmTile = 128 sub-elements the twelve planes of the tile, one after the other
//      (blk[(s / 128) 12 128 + q 128 + s % 128]) -- a wave's 64 lanes x 2 sub-elements read each of its
//      twelve 1 KiB pieces with one 16-byte load per lane, and the wave's block words are ONE contiguous
//      12 KiB run: 7 streams a launch (x, b and the blocks in, the sweep out) instead of 21.
// Measured (scripts/asm_probe.py, profiles/r05_e_asm_layouts.txt; 4 layouts x 2 plane gaps, two interleaved
// rounds, one process each): every variant 0.240-0.259 ms per launch = 5.4-5.9 TB/s, the spread between
// processes of one variant (their allocations' placement) as large as between variants -- the stream count
// is not what bounds it; 0.70-0.73 of 8 TB/s is ~93 % of the guide's measured 6.3 TB/s streaming copy.
// Then 12 (tiled, two tiles per wave: the best mean, 0.246 ms). Default 41 (round 5): the tiled blocks and the x / b
// pieces of a wave's tile all through LDS-DMA (global_load_lds_dwordx4, 18 wave-instructions of 1 KiB, no VGPR
// destination), 0.749-0.755 of 8 TB/s against 0.716-0.724 for 12 and 0.709-0.724 for the blocks alone through LDS
// (31), three interleaved process triples (profiles/r05_ad_asm_ldsdma.txt).
constexpr int kAsmTile = 128;
__device__ __forceinline__ int64_t asm_index(int layout, int64_t pitch, int q, int64_t s) {
    return layout == 0 ? q * pitch + s : (s / kAsmTile) * (12 * kAsmTile) + q * kAsmTile + (s % kAsmTile);
}

__global__ __launch_bounds__(kBlock) void k_build_blocks(const double *__restrict__ stc, double *__restrict__ blk,
                                                         int64_t pitch, int64_t N, int nsub_log2, int layout) {
    const int64_t s = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (s >= N) return;
    const double *r = stc + (s >> nsub_log2) * kStcStride;
#pragma unroll
    for (int q = 0; q < 9; ++q) blk[asm_index(layout, pitch, q, s)] = r[kStcA + q];
#pragma unroll
    for (int q = 0; q < 3; ++q) blk[asm_index(layout, pitch, 9 + q, s)] = r[kStcW + q];
}

// one adjacent pair s, s + 1 (s even) of the sweep from its loaded words
__device__ __forceinline__ void asm_pair(const double2 xv[3], const double2 bv[3], const double2 a[12],
                                         double *__restrict__ out, int64_t pitch, int64_t s) {
    StcF S0, S1;
#pragma unroll
    for (int q = 0; q < 9; ++q) { S0.A[q] = a[q].x; S1.A[q] = a[q].y; }
#pragma unroll
    for (int q = 0; q < 3; ++q) { S0.w[q] = a[9 + q].x; S1.w[q] = a[9 + q].y; }
    double x0[3] = {xv[0].x, xv[1].x, xv[2].x}, x1[3] = {xv[0].y, xv[1].y, xv[2].y};
    const double b0[3] = {bv[0].x, bv[1].x, bv[2].x}, b1[3] = {bv[0].y, bv[1].y, bv[2].y};
    sweep(S0, 0.0, b0, x0);
    sweep(S1, 0.0, b1, x1);
#pragma unroll
    for (int c = 0; c < 3; ++c) st2(out + c * pitch + s, make_double2(x0[c], x1[c]));
}

// LAYOUT 0: a thread per pair. LAYOUT 1: a wave per run of K tiles (K x 128 sub-elements), a lane takes pair
// `lane` of each tile, every load of the K tiles issued before the first sweep. (Measured, not kept: a resident
// grid whose waves walk the tiles w, w + W, ... with the next tile's loads in flight in a second register set --
// 206 VGPRs, two waves per SIMD -- 0.64-0.70 of 8 TB/s against this launch's 0.70-0.72, profiles/r05_aa_*.)
template <int LAYOUT, int K>
__global__ __launch_bounds__(kBlock) void k_sweep_assembled(const double *__restrict__ x, const double *__restrict__ b,
                                                            const double *__restrict__ blk, double *__restrict__ out,
                                                            int64_t pitch, int64_t npairs) {
    if constexpr (LAYOUT == 0) {
        const int64_t p = (int64_t)blockIdx.x * kBlock + threadIdx.x;
        if (p >= npairs) return;
        const int64_t s = 2 * p;
        double2 xv[3], bv[3], a[12];
#pragma unroll
        for (int c = 0; c < 3; ++c) { xv[c] = ld2(x + c * pitch + s); bv[c] = ld2(b + c * pitch + s); }
#pragma unroll
        for (int q = 0; q < 12; ++q) a[q] = ld2(blk + q * pitch + s);
        asm_pair(xv, bv, a, out, pitch, s);
    } else if constexpr (LAYOUT == 4) {
        // every stream through LDS-DMA: the twelve block pieces and the six x / b pieces of the wave's tile (18 KiB,
        // 18 wave-instructions, no VGPR destination); a partial last tile loads x and b into registers
        constexpr int NP = 18;
        __shared__ double LB[(kBlock / 64) * NP * kAsmTile];
        const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
        const int64_t tile = (int64_t)blockIdx.x * (kBlock / 64) + wv;
        const int64_t ntiles = (2 * npairs + kAsmTile - 1) / kAsmTile;
        if (tile >= ntiles) return;
        const int64_t s = tile * kAsmTile + 2 * lane;
        const bool full = (tile + 1) * kAsmTile <= 2 * npairs;
        double *l = LB + wv * NP * kAsmTile;
        const double *t = blk + tile * (12 * kAsmTile) + 2 * lane;
        constexpr int aux = (PAMG_NT & 1) ? 2 : 0;
#pragma unroll
        for (int q = 0; q < 12; ++q)
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)(t + q * kAsmTile),
                                             (__attribute__((address_space(3))) void *)(l + q * kAsmTile), 16, 0, aux);
        double2 xv[3], bv[3];
        if (full) {
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)(x + c * pitch + s),
                                                 (__attribute__((address_space(3))) void *)(l + (12 + c) * kAsmTile), 16, 0, aux);
                __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)(b + c * pitch + s),
                                                 (__attribute__((address_space(3))) void *)(l + (15 + c) * kAsmTile), 16, 0, aux);
            }
        } else if (s < 2 * npairs) {
#pragma unroll
            for (int c = 0; c < 3; ++c) { xv[c] = ld2(x + c * pitch + s); bv[c] = ld2(b + c * pitch + s); }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (s >= 2 * npairs) return;
        const double *lr = l + 2 * lane;
        double2 a[12];
#pragma unroll
        for (int q = 0; q < 12; ++q) a[q] = *reinterpret_cast<const double2 *>(lr + q * kAsmTile);
        if (full)
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                xv[c] = *reinterpret_cast<const double2 *>(lr + (12 + c) * kAsmTile);
                bv[c] = *reinterpret_cast<const double2 *>(lr + (15 + c) * kAsmTile);
            }
        asm_pair(xv, bv, a, out, pitch, s);
    } else if constexpr (LAYOUT == 3) {
        // the tiled blocks through LDS-DMA (global_load_lds_dwordx4: a plane piece of a tile is 64 lanes x 16 B, one
        // wave-instruction, no VGPR destination), x and b into registers; then each lane reads its 16 B of every
        // piece from LDS (lane-linear: conflict-free ds_read_b128)
        __shared__ double LB[(kBlock / 64) * K * 12 * kAsmTile];
        const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
        const int64_t w = (int64_t)blockIdx.x * (kBlock / 64) + wv;
        const int64_t ntiles = (2 * npairs + kAsmTile - 1) / kAsmTile;
        double2 xv[K][3], bv[K][3];
        int64_t sk[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int64_t tile = w * K + k;
            sk[k] = tile * kAsmTile + 2 * lane;
            if (tile >= ntiles) continue;
            const double *t = blk + tile * (12 * kAsmTile) + 2 * lane;
            double *l = LB + (wv * K + k) * 12 * kAsmTile;
#pragma unroll
            for (int q = 0; q < 12; ++q)
                __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)(t + q * kAsmTile),
                                                 (__attribute__((address_space(3))) void *)(l + q * kAsmTile), 16, 0,
                                                 (PAMG_NT & 1) ? 2 : 0);
            if (sk[k] < 2 * npairs)
#pragma unroll
                for (int c = 0; c < 3; ++c) { xv[k][c] = ld2(x + c * pitch + sk[k]); bv[k][c] = ld2(b + c * pitch + sk[k]); }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
        for (int k = 0; k < K; ++k) {
            if (sk[k] >= 2 * npairs) continue;
            const double *l = LB + (wv * K + k) * 12 * kAsmTile + 2 * lane;
            double2 a[12];
#pragma unroll
            for (int q = 0; q < 12; ++q) a[q] = *reinterpret_cast<const double2 *>(l + q * kAsmTile);
            asm_pair(xv[k], bv[k], a, out, pitch, sk[k]);
        }
    } else {
        const int64_t w = (int64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
        const int lane = threadIdx.x & 63;
        double2 xv[K][3], bv[K][3], a[K][12];
        int64_t sk[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            sk[k] = (w * K + k) * kAsmTile + 2 * lane;
            if (sk[k] >= 2 * npairs) continue;
            const double *t = blk + (w * K + k) * (12 * kAsmTile) + 2 * lane;
#pragma unroll
            for (int q = 0; q < 12; ++q) a[k][q] = ld2(t + q * kAsmTile);
#pragma unroll
            for (int c = 0; c < 3; ++c) { xv[k][c] = ld2(x + c * pitch + sk[k]); bv[k][c] = ld2(b + c * pitch + sk[k]); }
        }
#pragma unroll
        for (int k = 0; k < K; ++k)
            if (sk[k] < 2 * npairs) asm_pair(xv[k], bv[k], a[k], out, pitch, sk[k]);
    }
}

// Matrix-free form of the same sweep (the reference's own structure: one
// stencil per un_ele, ShapFun_unstruc.F90:304-335): 72 B per sub-element.
// (Measured, not kept: x and b through LDS-DMA, 0.737-0.753 of 8 TB/s against 0.747-0.772 with these register
// loads, profiles/r05_ae_face_pp_glds.txt -- unlike the assembled sweep's 18 streams, this sweep's six gain nothing.)
__global__ __launch_bounds__(kBlock) void k_sweep_stencil(const double *__restrict__ x, const double *__restrict__ b,
                                                          const double *__restrict__ stc, double *__restrict__ out,
                                                          int64_t pitch, int64_t npairs, int nsub_log2, double rdt) {
    const int64_t p = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (p >= npairs) return;
    const int64_t s = 2 * p;
    double2 xv[3], bv[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) { xv[c] = ld2(x + c * pitch + s); bv[c] = ld2(b + c * pitch + s); }
    Stc S;
    load_stc(stc + (s >> nsub_log2) * kStcStride, S);
    double x0[3] = {xv[0].x, xv[1].x, xv[2].x}, x1[3] = {xv[0].y, xv[1].y, xv[2].y};
    const double b0[3] = {bv[0].x, bv[1].x, bv[2].x}, b1[3] = {bv[0].y, bv[1].y, bv[2].y};
    sweep(S, rdt, b0, x0);
    sweep(S, rdt, b1, x1);
#pragma unroll
    for (int c = 0; c < 3; ++c) st2(out + c * pitch + s, make_double2(x0[c], x1[c]));
}

// FINDInv (matrix_inversion.F90:50-148), the reference's local block solve: Gauss-Jordan
// on [A | I] without pivoting, a zero pivot repaired by adding the first lower row with a
// nonzero entry in that column (:75-86) -- the search gives up at the first zero entry
// (:87-92) -- errorflag -1 and inverse 0 for a singular matrix (:94-102). Column-major
// n x n, the reference's operation order (bitwise equal to it, tests/test_block_inverse.py).
template <int N>
__device__ __forceinline__ int findinv(const double *__restrict__ A, double *__restrict__ inv) {
    double ag[N][2 * N];
#pragma unroll
    for (int i = 0; i < N; ++i)
#pragma unroll
        for (int j = 0; j < 2 * N; ++j) ag[i][j] = j < N ? A[i + j * N] : (j - N == i ? 1.0 : 0.0);
    int err = 0;
#pragma unroll
    for (int k = 0; k < N - 1; ++k) {
        if (ag[k][k] == 0) {
            bool found = false;
#pragma unroll
            for (int i = k + 1; i < N; ++i) {
                if (found || err) continue;
                if (ag[i][k] != 0) {
#pragma unroll
                    for (int j = 0; j < 2 * N; ++j) ag[k][j] = ag[k][j] + ag[i][j];
                    found = true;
                } else {
                    err = -1;   // :87-92: the first zero entry ends the search
                }
            }
        }
        if (err) break;
#pragma unroll
        for (int j = k + 1; j < N; ++j) {
            const double m = ag[j][k] / ag[k][k];
#pragma unroll
            for (int i = k; i < 2 * N; ++i) ag[j][i] = ag[j][i] - m * ag[k][i];
        }
    }
    if (!err) {
#pragma unroll
        for (int i = 0; i < N; ++i)
            if (ag[i][i] == 0) err = -1;
    }
    if (err) {
#pragma unroll
        for (int q = 0; q < N * N; ++q) inv[q] = 0.0;
        return err;
    }
#pragma unroll
    for (int i = 0; i < N; ++i) {
        const double m = ag[i][i];
#pragma unroll
        for (int j = i; j < 2 * N; ++j) ag[i][j] = ag[i][j] / m;
    }
#pragma unroll
    for (int k = N - 2; k >= 0; --k)
#pragma unroll
        for (int i = 0; i <= k; ++i) {
            const double m = ag[i][k + 1];
#pragma unroll
            for (int j = k; j < 2 * N; ++j) ag[i][j] = ag[i][j] - ag[k + 1][j] * m;
        }
#pragma unroll
    for (int i = 0; i < N; ++i)
#pragma unroll
        for (int j = 0; j < N; ++j) inv[i + j * N] = ag[i][j + N];
    return 0;
}

// one matrix per thread
template <int N>
__global__ __launch_bounds__(64) void k_block_inverse(const double *__restrict__ A, double *__restrict__ inv,
                                                      int *__restrict__ err, int64_t nb) {
    const int64_t q = (int64_t)blockIdx.x * 64 + threadIdx.x;
    if (q >= nb) return;
    double a[N * N], o[N * N];
#pragma unroll
    for (int i = 0; i < N * N; ++i) a[i] = A[q * N * N + i];
    err[q] = findinv<N>(a, o);
#pragma unroll
    for (int i = 0; i < N * N; ++i) inv[q * N * N + i] = o[i];
}

// the exact local solve of the smoother's operator: per un_ele, A_e = (1/dt) M + Kd
// (get_A_x, transport_tri_semi.F90:412-448, as an assembled block; matrices.F90 block-CSR
// with one block per block-row) and its FINDInv inverse, column-major at Ainv + 9 u
__global__ __launch_bounds__(kBlock) void k_block_ops(const double *__restrict__ stc, double rdt,
                                                      double *__restrict__ Ainv, int *__restrict__ err, int U) {
    const int u = blockIdx.x * kBlock + threadIdx.x;
    if (u >= U) return;
    const double *r = stc + (int64_t)u * kStcStride;
    double a[9], o[9];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) a[i + 3 * j] = rdt * r[kStcM + 3 * i + j] + r[kStcK + 3 * i + j];
    err[u] = findinv<3>(a, o);
#pragma unroll
    for (int q = 0; q < 9; ++q) Ainv[9 * (int64_t)u + q] = o[q];
}

// direct solve of a level: tnew = tnew_nonlin = A_e^-1 RHS per sub-element
__global__ __launch_bounds__(kBlock) void k_block_solve(double *__restrict__ T, double *__restrict__ TNN,
                                                        const double *__restrict__ RHS,
                                                        const double *__restrict__ Ainv, int64_t pitch, int64_t N,
                                                        int nsub_log2) {
    const int64_t s = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (s >= N) return;
    const double *ai = Ainv + 9 * (s >> nsub_log2);
    const double b[3] = {RHS[s], RHS[pitch + s], RHS[2 * pitch + s]};
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const double x = ai[i] * b[0] + ai[i + 3] * b[1] + ai[i + 6] * b[2];
        T[i * pitch + s] = x;
        TNN[i * pitch + s] = x;
    }
}

inline unsigned grid_for(int64_t n) { return (unsigned)((n + kBlock - 1) / kBlock); }
inline int log2i(int v) { int r = 0; while ((1 << r) < v) ++r; return r; }

}  // namespace

hipError_t launch_smooth(hipStream_t s, const Level &L, const double *src, int sweeps, int solver, double rdt,
                         double omega, double *tov, double *tovo) {
    const int64_t npairs = L.N / 2;
    if (npairs == 0 || sweeps <= 0) return hipSuccess;
    const HaloPlan &P = L.halo;
    HaloArgs H{P.d_hsub, P.d_hface, P.d_bcv, P.d_told_halo, tov, tovo, P.d_send, 1 << L.isplit};
    // diagnostics build only (make PAMG_STAMPS=1): the halo words not written (wrong results) or the non-uniform
    // instance, for A/B timing of the fused forms
    static const bool diag_nohalo = PAMG_STAMPS && getenv("PAMG_DIAG_NOHALO") != nullptr;
    static const bool diag_nouniform = PAMG_STAMPS && getenv("PAMG_DIAG_NOUNIFORM") != nullptr;
    if (diag_nohalo) H.hsub = nullptr;
    const int lg = log2i(L.nsub);
    const dim3 g(grid_for(npairs)), b(kBlock);
#define PAMG_SM(R, U, ST) \
    hipLaunchKernelGGL((k_smooth<R, U, ST>), g, b, 0, s, src, L.T, L.TNN, L.RHS, L.stc, L.pitch, npairs, lg, sweeps, \
                       rdt, omega, H)
    const bool uni = L.nsub >= 128 && !diag_nouniform;
    if (solver == 2) PAMG_SM(true, false, Stc);
    else if (L.arith == 1) { if (uni) PAMG_SM(false, true, StcF); else PAMG_SM(false, false, StcF); }
    else if (uni) PAMG_SM(false, true, Stc);
    else PAMG_SM(false, false, Stc);
#undef PAMG_SM
    return hipGetLastError();
}

hipError_t launch_residual(hipStream_t s, const Level &L, double rdt, bool neg) {
    const int64_t npairs = L.N / 2;
    if (npairs == 0) return hipSuccess;
#define PAMG_RES(ST, NEG)                                                                                          \
    hipLaunchKernelGGL((k_residual<ST, NEG>), dim3(grid_for(npairs)), dim3(kBlock), 0, s, L.T, L.RHS, L.RES, L.stc, \
                       L.pitch, npairs, log2i(L.nsub), rdt)
    if (L.arith == 1) { if (neg) PAMG_RES(StcF, true); else PAMG_RES(StcF, false); }
    else if (neg) PAMG_RES(Stc, true);
    else PAMG_RES(Stc, false);
#undef PAMG_RES
    return hipGetLastError();
}

hipError_t launch_interp_add(hipStream_t s, const Level &fine, const Level &coarse) {
    if (coarse.N == 0) return hipSuccess;
    hipLaunchKernelGGL(k_interp_add, dim3(grid_for(4 * coarse.N)), dim3(kBlock), 0, s, fine.T, coarse.T, fine.pitch,
                       coarse.pitch, coarse.N);
    return hipGetLastError();
}

// aligned tiles of 1024 fine sub-elements (each carries its own 256 coarse ones, Level::pos);
// LDS = 3 * 1024 * 8 B = 24 KiB
constexpr int kTileLog2 = 10;

hipError_t launch_restrict(hipStream_t s, const Level &fine, const Level &coarse, int U, double *out) {
    double *dst = out ? out : coarse.RHS;
    (void)U;
    if (coarse.N == 0) return hipSuccess;
    const int tl = kTileLog2;
    const unsigned grid = (unsigned)((fine.N + (1ll << tl) - 1) >> tl);
    hipLaunchKernelGGL(k_restrict_tile, dim3(grid), dim3(kBlock), (size_t)3 * 8 << tl, s, fine.RES, dst, fine.pitch,
                       coarse.pitch, fine.N, tl);
    return hipGetLastError();
}

hipError_t launch_restrict_residual(hipStream_t s, const Level &fine, const Level &coarse, double rdt) {
    if (fine.N == 0) return hipSuccess;
    // aligned tiles of 1024 fine sub-elements (each with its own coarse sub-elements, Level::pos)
    const int tl = kTileLog2;
    const unsigned grid = (unsigned)((fine.N + (1ll << tl) - 1) >> tl);
    const size_t lds = (size_t)3 * 8 << tl;
    const int lg = log2i(fine.nsub);
#define PAMG_RR(U, IT, ST)                                                                                      \
    hipLaunchKernelGGL((k_restrict_residual<U, IT, ST>), dim3(grid), dim3(kBlock), lds, s, fine.T, fine.RHS,       \
                       fine.RES, coarse.RHS, fine.stc, fine.pitch, coarse.pitch, fine.N, lg, rdt)
    if (fine.arith == 1) { if (fine.nsub >= 128) PAMG_RR(true, 2, StcF); else PAMG_RR(false, 2, StcF); }
    else if (fine.nsub >= 128) PAMG_RR(true, 2, Stc);
    else PAMG_RR(false, 2, Stc);
#undef PAMG_RR
    return hipGetLastError();
}

hipError_t launch_prolong(hipStream_t s, const Level &fine, const Level &coarse, bool write_tnn) {
    if (coarse.N == 0) return hipSuccess;
    const int tl = kTileLog2;
    const unsigned grid = (unsigned)((fine.N + (1ll << tl) - 1) >> tl);
    hipLaunchKernelGGL(k_prolong_tile, dim3(grid), dim3(kBlock), (size_t)3 * 8 << tl, s, fine.T, fine.TNN, coarse.T,
                       fine.pitch, coarse.pitch, fine.N, tl, write_tnn ? 1 : 0);
    return hipGetLastError();
}

hipError_t launch_rhs(hipStream_t s, const Level &L, double rdt, int start_of_step, bool told_halo) {
    if (L.N == 0) return hipSuccess;
    if ((L.N & 1) || (L.pitch & 1) || !L.SRC) return hipErrorInvalidValue;   // pairs of one un_ele, 16-byte aligned
    hipLaunchKernelGGL(k_rhs, dim3(grid_for(L.N / 2)), dim3(kBlock), 0, s, L.T, L.TOLD, L.TNN, L.RHS, L.SRC, L.stc,
                       L.pitch, L.N, log2i(L.nsub), rdt, start_of_step, L.halo.d_hsub, L.halo.d_hface,
                       (told_halo && start_of_step && L.halo.d_hface && L.halo.d_hsub) ? L.halo.d_told_halo : nullptr);
    return hipGetLastError();
}

hipError_t launch_source(hipStream_t s, const Level &L, const double *geo1, double k) {
    if (L.N == 0) return hipSuccess;
    if (!L.SRC) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_source, dim3(grid_for(L.N)), dim3(kBlock), 0, s, L.SRC, L.stc, geo1, L.subinfo, L.pitch, L.N,
                       log2i(L.nsub), k);
    return hipGetLastError();
}

hipError_t launch_halo_unpack(hipStream_t s, const Level &L, double *tov, double *tovo) {
    const HaloPlan &P = L.halo;
    const int n = (int)P.recv_dst.size();
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_halo_unpack, dim3(grid_for(n)), dim3(kBlock), 0, s, P.d_recv, P.d_recv_dst, n, tov, tovo);
    return hipGetLastError();
}

hipError_t launch_halo_unpack3(hipStream_t s, const Level &L, double *tov) {
    const HaloPlan &P = L.halo;
    const int n = (int)P.recv_dst.size();
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_halo_unpack3, dim3(grid_for(n)), dim3(kBlock), 0, s, P.d_recv3, P.d_recv_dst, n, tov);
    return hipGetLastError();
}

hipError_t launch_copy(hipStream_t s, const double *src, double *dst, int64_t n) {
    const int64_t n2 = n / 2;   // planes are multiples of 64 doubles
    if (n2 == 0) return hipSuccess;
    const unsigned g = (unsigned)std::min<int64_t>((n2 + kBlock - 1) / kBlock, 8192);
    hipLaunchKernelGGL(k_copy, dim3(g), dim3(kBlock), 0, s, src, dst, n2);
    return hipGetLastError();
}

hipError_t launch_told_halo(hipStream_t s, const Level &L, int U) {
    const HaloPlan &P = L.halo;
    if (P.n_told == 0 || U == 0) return hipSuccess;
    const int m = 1 << L.isplit;
    hipLaunchKernelGGL(k_told_halo, dim3(grid_for((int64_t)U * 3 * m)), dim3(kBlock), 0, s, L.TOLD, L.pitch,
                       P.d_hface, P.d_surf, P.d_told_halo, U, m, log2i(L.nsub));
    return hipGetLastError();
}

hipError_t launch_overlap_static(hipStream_t s, const Level &L, int U, double *tov, double *tovo, double *send,
                                 bool from_told) {
    const HaloPlan &P = L.halo;
    if (U == 0 || P.d_hface == nullptr) return hipSuccess;
    const int m = 1 << L.isplit;
    HaloArgs H{P.d_hsub, P.d_hface, P.d_bcv, P.d_told_halo, tov, tovo, send ? send : P.d_send, m};
    hipLaunchKernelGGL(k_overlap_static, dim3(grid_for((int64_t)U * 3 * m)), dim3(kBlock), 0, s, H, P.d_surf, U,
                       from_told ? L.TOLD : nullptr, L.pitch, log2i(L.nsub));
    return hipGetLastError();
}

hipError_t launch_block_inverse(hipStream_t s, int n, int64_t nb, const double *A, double *inv, int *err) {
    if (nb == 0) return hipSuccess;
    const unsigned g = (unsigned)((nb + 63) / 64);
    switch (n) {
        case 1: hipLaunchKernelGGL(k_block_inverse<1>, dim3(g), dim3(64), 0, s, A, inv, err, nb); break;
        case 2: hipLaunchKernelGGL(k_block_inverse<2>, dim3(g), dim3(64), 0, s, A, inv, err, nb); break;
        case 3: hipLaunchKernelGGL(k_block_inverse<3>, dim3(g), dim3(64), 0, s, A, inv, err, nb); break;
        case 4: hipLaunchKernelGGL(k_block_inverse<4>, dim3(g), dim3(64), 0, s, A, inv, err, nb); break;
        case 5: hipLaunchKernelGGL(k_block_inverse<5>, dim3(g), dim3(64), 0, s, A, inv, err, nb); break;
        case 6: hipLaunchKernelGGL(k_block_inverse<6>, dim3(g), dim3(64), 0, s, A, inv, err, nb); break;
        case 7: hipLaunchKernelGGL(k_block_inverse<7>, dim3(g), dim3(64), 0, s, A, inv, err, nb); break;
        case 8: hipLaunchKernelGGL(k_block_inverse<8>, dim3(g), dim3(64), 0, s, A, inv, err, nb); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_block_ops(hipStream_t s, const Level &L, int U, double rdt, double *Ainv, int *err) {
    if (U == 0) return hipSuccess;
    hipLaunchKernelGGL(k_block_ops, dim3(grid_for(U)), dim3(kBlock), 0, s, L.stc, rdt, Ainv, err, U);
    return hipGetLastError();
}

hipError_t launch_block_solve(hipStream_t s, const Level &L, const double *Ainv) {
    if (L.N == 0) return hipSuccess;
    hipLaunchKernelGGL(k_block_solve, dim3(grid_for(L.N)), dim3(kBlock), 0, s, L.T, L.TNN, L.RHS, Ainv, L.pitch, L.N,
                       log2i(L.nsub));
    return hipGetLastError();
}

hipError_t launch_to_soa(hipStream_t s, const Level &L, const double *aos, double *soa) {
    if (L.N == 0) return hipSuccess;
    hipLaunchKernelGGL(k_to_soa, dim3(grid_for(L.N)), dim3(kBlock), 0, s, aos, soa, L.d_pos, L.N, L.pitch,
                       log2i(L.nsub));
    return hipGetLastError();
}

hipError_t launch_to_aos(hipStream_t s, const Level &L, const double *soa, double *aos) {
    if (L.N == 0) return hipSuccess;
    hipLaunchKernelGGL(k_to_aos, dim3(grid_for(L.N)), dim3(kBlock), 0, s, soa, aos, L.d_pos, L.N, L.pitch,
                       log2i(L.nsub));
    return hipGetLastError();
}

// the assembled blocks are tiled (layout 1 of the note above k_build_blocks), swept by k_sweep_assembled<4, 1>
constexpr int kAsmLayout = 1;

size_t asm_blocks_doubles(const Level &L) {
    return 12 * (size_t)((L.pitch + kAsmTile - 1) / kAsmTile * kAsmTile);
}

hipError_t launch_build_blocks(hipStream_t s, const Level &L, double rdt) {
    (void)rdt;   // the blocks are the records' kStcA words, assembled with rdt on the host
    hipLaunchKernelGGL(k_build_blocks, dim3(grid_for(L.N)), dim3(kBlock), 0, s, L.stc, L.blocks, L.pitch, L.N,
                       log2i(L.nsub), kAsmLayout);
    return hipGetLastError();
}

hipError_t launch_sweep_assembled(hipStream_t s, const Level &L, double *out, double rdt) {
    (void)rdt;
    if (L.N % 2) return hipErrorInvalidValue;
    const int64_t npairs = L.N / 2;
    // tiled, every stream of a wave's tile of 128 sub-elements through LDS-DMA (the other layouts and tilings of
    // the note above k_build_blocks measured slower and are removed)
    const int64_t ntiles = (L.N + kAsmTile - 1) / kAsmTile;
    const unsigned g4 = (unsigned)((ntiles + kBlock / 64 - 1) / (kBlock / 64));
    hipLaunchKernelGGL((k_sweep_assembled<4, 1>), dim3(g4), dim3(kBlock), 0, s, L.TNN, L.RHS, L.blocks, out, L.pitch, npairs);
    return hipGetLastError();
}

hipError_t launch_sweep_stencil(hipStream_t s, const Level &L, double *out, double rdt) {
    const int64_t npairs = L.N / 2;
    hipLaunchKernelGGL(k_sweep_stencil, dim3(grid_for(npairs)), dim3(kBlock), 0, s, L.TNN, L.RHS, L.stc, out,
                       L.pitch, npairs, log2i(L.nsub), rdt);
    return hipGetLastError();
}

}  // namespace pamg
