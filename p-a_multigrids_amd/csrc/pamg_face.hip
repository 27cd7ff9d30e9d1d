// The face-coupled operator (pamg_params.op = 1) on gfx950.
//
// A x of a sub-element adds to the reference's element operator (1/dt) M x + Kd x the
// interior-penalty diffusion surface terms its smoother and residual leave commented out
// (transport_tri_semi.F90:619-688, :789-857; add_diffusion_surf, matrices.F90:66-117): per face
// f with nodes (a, b) and the neighbour's values (ya, yb) at those nodes,
//   ds_a += w_f ((2 x_a + x_b) - 2 ya - yb),  ds_b += w_f ((x_a + 2 x_b) - ya - 2 yb),
//   w_f = k / delta_x |e_f| / 6 (the P1 edge mass matrix), D_a += 2 w_f (get_diagonal's surface
// term, :481-486). Inner neighbours are read from the level's field; across an un_ele face the
// values come from t_overlap, the halo update_overlaps writes at the start of every sweep (:555)
// -- with several ranks, after the exchange: the first consumer of the halo. A sweep is
// red-black Gauss-Seidel on the up / down sub-elements (solver 3: every inner neighbour of an up
// sub-element is a down one) or Jacobi (solver 1). The operation order is the oracle's
// (oracle/pamg_oracle.c face_terms / face_sweep), so the results are bitwise its own. The forms:
// per-colour kernels (k_face), one launch per sweep on LDS tiles (k_face_sweep), and a whole
// smoother call in one cooperative launch for a level that fits on-chip (k_face_chain); the face
// V-cycle (pamg_api.cpp vcycle_face_fused) strings them together. A grid-stride form that kept the
// next tile in flight (two workgroups per CU) measured 5 % slower than one launch per tile and was
// dropped (profiles/r03_c_face_ab.txt).
#include <hip/hip_runtime.h>

#include <map>
#include <mutex>

#include "pamg_device.h"
#include "pamg_internal.h"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

namespace pamg {
namespace {

using namespace detail;

// face_nodes, 0-based (:142-147), and the un_ele face under sub-element face f -- compile-time, so that
// every index derived from them in the unrolled face loops is a constant (a register array or record
// indexed at run time goes to scratch)
__host__ __device__ constexpr int fnode(int fi, int k) { return fi == 0 ? (k ? 2 : 0) : fi == 1 ? (k ? 1 : 2) : (k ? 0 : 1); }
__host__ __device__ constexpr int fmface(int fi) { return fi == 0 ? 1 : fi == 1 ? 3 : 2; }

// halo words of level L from its tnew, the sweep start: copy = tnew := tnew_nonlin first (:550)
__global__ __launch_bounds__(kBlock) void k_face_halo(double *T, const double *__restrict__ TNN, int64_t pitch,
                                                      int64_t npairs, int nsub_log2, HaloArgs H, int copy) {
    const int64_t p = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (p >= npairs) return;
    const int64_t s = 2 * p;
    HaloPre hp;
    halo_prefetch(H, s, s >> nsub_log2, nsub_log2, hp);
    if (!copy && !hp.any) return;   // the words-only form reads just the pairs that have words
    double2 v[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        v[c] = ld2((copy ? TNN : T) + c * pitch + s);
        if (copy) st2(T + c * pitch + s, v[c]);
    }
    const double p0[3] = {v[0].x, v[1].x, v[2].x}, p1[3] = {v[0].y, v[1].y, v[2].y};
    halo_write(H, hp, p0, p1);
}

// the words-only refresh (launch_face_halo(copy = false)'s words) over the sub-elements that have
// words: thread i -> un_ele i / nb, position bpos[i % nb]; the told words from the compact told halo
// (halo_prefetch's rule), every word through halo_face as k_face_halo writes it
__global__ __launch_bounds__(kBlock) void k_face_words(const double *__restrict__ T, int64_t pitch, HaloArgs H,
                                                       const int *__restrict__ bpos, int nb, int64_t nwork,
                                                       int nsub_log2) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= nwork) return;
    const int64_t u = i / nb;
    const int p = bpos[i - u * nb];
    const int64_t s = (u << nsub_log2) + p;
    HaloPre P;
    P.hs0 = H.hsub[p];
    P.r1 = H.hface[3 * u];
    P.r2 = H.hface[3 * u + 1];
    P.r3 = H.hface[3 * u + 2];
    double t[3], to[3] = {0.0, 0.0, 0.0};
#pragma unroll
    for (int c = 0; c < 3; ++c) t[c] = T[c * pitch + s];
    const int e = told_entry(P, P.hs0);
    if (e >= 0)
#pragma unroll
        for (int c = 0; c < 3; ++c) to[c] = H.told[3 * (int64_t)e + c];
    if (P.hs0.x) halo_face<true, true>(H, P.r1, 1, P.hs0.x, t, to);
    if (P.hs0.y) halo_face<true, true>(H, P.r2, 2, P.hs0.y, t, to);
    if (P.hs0.z) halo_face<true, true>(H, P.r3, 3, P.hs0.z, t, to);
}

// The operator record of one un_ele as face_apply reads it: the element stencil, the face weights
// w_f (inner faces 0..2 by sub-element face, then the un_ele faces 1..3) and the un_ele faces' node
// selectors (fsx) under sub-element faces 0..2
struct FaceRec {
    Stc S;
    double w[6];
    int sx[3];
};

__device__ __forceinline__ void load_face_rec(const double *__restrict__ stc, const double *__restrict__ fface,
                                              const int *__restrict__ fsx, int64_t u, FaceRec &R) {
    load_stc(stc + u * kStcStride, R.S);
#pragma unroll
    for (int q = 0; q < 6; ++q) R.w[q] = fface[u * kFaceStride + q];
#pragma unroll
    for (int fi = 0; fi < 3; ++fi) R.sx[fi] = fsx[4 * u + fmface(fi) - 1];
}

// the sub-element's pattern of inner faces (selects omega / D_i, kFaceWD)
__device__ __forceinline__ int face_pattern(int4 nb) { return (nb.x >= 0) | ((nb.y >= 0) << 1) | ((nb.z >= 0) << 2); }

// face_point's arithmetic from a loaded record and the neighbours' values: yf(fi, c) = component c of the
// neighbour across sub-element face fi (the inner neighbour's value, or slot -nb of the halo snapshot of
// un_ele face fmface(fi)); wd(i): omega / D_i of the sub-element's pattern
template <int MODE, class YF, class WD>
__device__ __forceinline__ void face_core(const FaceRec &R, const double x[3], const double b[3], int4 nb, const YF &yf,
                                          const WD &wd, int level1, double rdt, double out[3]) {
    double A[3];
    apply_A(R.S, rdt, x, A);
    double ds[3] = {0.0, 0.0, 0.0};
    const int nbf[3] = {nb.x, nb.y, nb.z};
#pragma unroll
    for (int fi = 0; fi < 3; ++fi) {
        const int a = fnode(fi, 0), bb = fnode(fi, 1);
        double ya, yb, wf;
        if (nbf[fi] >= 0) {   // inner neighbour: its nodes at my face nodes a, b are its b, a
            ya = yf(fi, bb);
            yb = yf(fi, a);
            wf = R.w[fi];
        } else {              // across the un_ele face: the halo (t_overlap slot sp)
            const int mface = fmface(fi), sx = R.sx[fi];
            if (!level1 && (sx & 16)) {
                ya = 0.0;     // coarse levels carry the error equation: homogeneous boundary data
                yb = 0.0;
            } else {
                ya = yf(fi, (sx & 3) - 1);
                yb = yf(fi, ((sx >> 2) & 3) - 1);
            }
            wf = R.w[3 + mface - 1];
        }
        ds[a] = ds[a] + wf * (((2.0 * x[a] + x[bb]) - 2.0 * ya) - yb);
        ds[bb] = ds[bb] + wf * (((x[a] + 2.0 * x[bb]) - ya) - 2.0 * yb);
    }
    // omega / D_i of the sub-element's pattern of inner faces (kFaceWD: D accumulated and divided on
    // the host in the oracle's order -- no division here)
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const double ai = A[i] + ds[i];
        if (MODE <= 2) out[i] = x[i] + wd(i) * (b[i] - ai);
        else if (MODE == 3) out[i] = ai - b[i];
        else out[i] = b[i] - ai;
    }
}

// face_core's arithmetic with the neighbours read from the tile (xin(c, q): component c at un_ele position
// q) and the halo snapshot (hv(u, mface, sp, c)) -- written out rather than through face_core's accessor,
// which put the record in scratch in the tile kernels; the same operations in the same order (the
// two-sweep passes' ghost updates use face_core: tests/test_face_operator.py holds them bitwise equal)
template <int MODE, class XIN, class HV, class WD>
__device__ __forceinline__ void face_apply(const FaceRec &R, const XIN &xin, const double x[3], const double b[3],
                                           int4 nb, int64_t u, const HV &hv, const WD &wd, int level1, double rdt,
                                           double out[3]) {
    double A[3];
    apply_A(R.S, rdt, x, A);
    double ds[3] = {0.0, 0.0, 0.0};
    const int nbf[3] = {nb.x, nb.y, nb.z};
#pragma unroll
    for (int fi = 0; fi < 3; ++fi) {
        const int a = fnode(fi, 0), bb = fnode(fi, 1);
        double ya, yb, wf;
        if (nbf[fi] >= 0) {   // inner neighbour: its nodes at my face nodes a, b are its b, a
            ya = xin(bb, nbf[fi]);
            yb = xin(a, nbf[fi]);
            wf = R.w[fi];
        } else {              // across the un_ele face: the halo (t_overlap slot sp)
            const int mface = fmface(fi), sx = R.sx[fi];
            if (!level1 && (sx & 16)) {
                ya = 0.0;     // coarse levels carry the error equation: homogeneous boundary data
                yb = 0.0;
            } else {
                ya = hv(u, mface, -nbf[fi], (sx & 3) - 1);
                yb = hv(u, mface, -nbf[fi], ((sx >> 2) & 3) - 1);
            }
            wf = R.w[3 + mface - 1];
        }
        ds[a] = ds[a] + wf * (((2.0 * x[a] + x[bb]) - 2.0 * ya) - yb);
        ds[bb] = ds[bb] + wf * (((x[a] + 2.0 * x[bb]) - ya) - 2.0 * yb);
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const double ai = A[i] + ds[i];
        if (MODE <= 2) out[i] = x[i] + wd(i) * (b[i] - ai);
        else if (MODE == 3) out[i] = ai - b[i];
        else out[i] = b[i] - ai;
    }
}

// One sub-element of the face-coupled operator (the oracle's face_terms / face_sweep order):
// MODE <= 2 the smoother update x_i + omega / D_i (b_i - (A x)_i), MODE 3 / 4 the residual
// A x - b / b - A x. x: the sub-element's values; xin(c, q): component c of the inner neighbour
// at un_ele position q; tov: the halo snapshot (t_overlap) the sweep reads.
// hv(u, mface, sp, k): component k of slot sp of t_overlap(:, mface) of un_ele u, the halo snapshot
// the sweep reads (global memory, or the persistent chain's LDS image of it)
template <int MODE, class XIN, class HV>
__device__ __forceinline__ void face_point(const XIN &xin, const double x[3], const double b[3], int4 nb, int64_t u,
                                           const double *__restrict__ stc, const double *__restrict__ fface,
                                           const int *__restrict__ fsx, const HV &hv, int level1, double rdt,
                                           double omega, double out[3]) {
    (void)omega;
    FaceRec R;
    load_face_rec(stc, fface, fsx, u, R);
    const double *wd = fface + u * kFaceStride + kFaceWD + 3 * face_pattern(nb);
    face_apply<MODE>(R, xin, x, b, nb, u, hv, [&](int i) { return wd[i]; }, level1, rdt, out);
}

// MODE 0 / 1: one colour of a red-black sweep (up / down sub-elements), X = OUT = tnew_nonlin;
// MODE 2: a Jacobi sweep, X = tnew, OUT = tnew_nonlin; MODE 3 / 4: residual A X - RHS / RHS - A X.
// UNI: every wave lies inside one un_ele (nsub >= 64): its operator and face records come through
// the scalar unit (one fetch per wave instead of one per lane)
template <int MODE, bool UNI>
__global__ __launch_bounds__(kBlock) void k_face(const double *X, double *OUT, const double *__restrict__ RHS,
                                                 const double *__restrict__ stc, const int4 *__restrict__ fnb,
                                                 const double *__restrict__ fface, const int *__restrict__ fsx,
                                                 const double *__restrict__ tov, int64_t pitch, int64_t N,
                                                 int nsub_log2, int slots, int level1, double rdt, double omega) {
    const int64_t s = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (s >= N) return;
    int64_t u = s >> nsub_log2;
    if (UNI) u = __builtin_amdgcn_readfirstlane((int)u);
    const int64_t base = u << nsub_log2;
    const int4 nb = fnb[s & ((1ll << nsub_log2) - 1)];
    if ((MODE == 0 && !nb.w) || (MODE == 1 && nb.w)) return;
    double x[3], b[3], r[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        x[c] = X[c * pitch + s];
        b[c] = RHS[c * pitch + s];
    }
    auto xin = [&](int c, int q) { return X[c * pitch + base + q]; };
    auto hv = [&](int64_t uu, int mf, int sp, int k) { return tov[uu * slots * 3 + (int64_t)(mf - 1) * slots + (sp - 1) * 3 + k]; };
    face_point<MODE>(xin, x, b, nb, u, stc, fface, fsx, hv, level1, rdt, omega, r);
#pragma unroll
    for (int i = 0; i < 3; ++i) OUT[i * pitch + s] = r[i];
}

// One whole smoother sweep on a tile of TS sub-elements (whole un_eles; NT threads, TS / NT
// sub-elements each), one launch instead of the halo refresh and two colour launches: the leg
// copy tnew := tnew_nonlin (:550), the sweep itself -- red-black (RB: up sub-elements, then down
// ones, the iterate in LDS) or Jacobi -- from the halo snapshot `tin`, tnew_nonlin stored, and,
// unless this is the call's last sweep, the halo words the NEXT sweep reads (update_overlaps,
// :555, from the new tnew_nonlin that its :550 copies into tnew) written through `Hn` into the
// other t_overlap buffer. Single domain only (a partition's halo crosses ranks between sweeps).
// tnew is rewritten by every sweep's :550 before anything reads it, so only the call's last
// sweep stores it (store 1: tnew_nonlin and tnew from the sweep's start; the call's first copy
// comes from the halo refresh before it). store 2 is the last executed sweep of a call whose final
// sweep is dead (its tnew_nonlin is overwritten unread inside a fused V-cycle): it
// stores its result as tnew -- the dead sweep's :550 -- and not tnew_nonlin, and its next-halo
// words are the dead sweep's :555 ones. store 0 stores tnew_nonlin only.
// Every sub-element's operations are face_point's, so the result is bitwise the per-colour
// kernels' (and the oracle's).
// (waves per SIMD: 6 for the wave-uniform 1024-tiles, 72-76 VGPRs; the others spill there)
#ifndef PAMG_FACE_WAVES
#define PAMG_FACE_WAVES 6
#endif
template <int TS, int NT, bool UNI, bool RB>
__global__ __launch_bounds__(NT, (UNI && TS <= 1024) ? PAMG_FACE_WAVES : 1) void k_face_sweep(double *T, double *TNN, const double *SRC, const double *__restrict__ RHS,
                                                   const double *__restrict__ stc, const int4 *__restrict__ fnb,
                                                   const double *__restrict__ fface, const int *__restrict__ fsx,
                                                   const double *__restrict__ tin, HaloArgs Hn, int next_halo, int store,
                                                   int64_t pitch, int64_t N, int nsub_log2, int slots, int level1,
                                                   double rdt, double omega) {
    constexpr int PER = TS / NT;
    __shared__ double X[3][TS];
    const int t = threadIdx.x;
    const int64_t s0 = (int64_t)blockIdx.x * TS;
    const int64_t nsm = (1ll << nsub_log2) - 1;
    double b[PER][3];   // the RHS and neighbour records of the thread's sub-elements, read once
    int4 nbr[PER];
#pragma unroll
    for (int k = 0; k < PER; ++k) {   // tnew := tnew_nonlin (:550); the iterate into LDS
        const int j = t + NT * k;
        const int64_t s = s0 + j < N ? s0 + j : s0;
        nbr[k] = fnb[s & nsm];
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            const double v = SRC[c * pitch + s];
            b[k][c] = RHS[c * pitch + s];
            X[c][j] = v;
            if (store == 1 && SRC != T && s0 + j < N) T[c * pitch + s] = v;
        }
    }
    __syncthreads();
    // one colour (0 up, 1 down) or the Jacobi sweep (2) of the thread's sub-elements
    auto pass = [&](auto mc) {
        constexpr int MODE = decltype(mc)::value;
        double r[PER][3];
        bool on[PER];
#pragma unroll
        for (int k = 0; k < PER; ++k) {
            const int j = t + NT * k;
            const int64_t s = s0 + j;
            on[k] = false;
            if (s >= N) continue;
            int64_t u = s >> nsub_log2;
            if (UNI) u = __builtin_amdgcn_readfirstlane((int)u);
            const int4 nb = nbr[k];
            if ((MODE == 0 && !nb.w) || (MODE == 1 && nb.w)) continue;
            on[k] = true;
            const int jb = (int)((u << nsub_log2) - s0);   // the un_ele's first tile position
            double x[3];
#pragma unroll
            for (int c = 0; c < 3; ++c) x[c] = X[c][j];
            auto xin = [&](int c, int q) { return X[c][jb + q]; };
            auto hv = [&](int64_t uu, int mf, int sp, int kk) {
                return tin[uu * slots * 3 + (int64_t)(mf - 1) * slots + (sp - 1) * 3 + kk];
            };
            face_point<MODE>(xin, x, b[k], nb, u, stc, fface, fsx, hv, level1, rdt, omega, r[k]);
            // a colour's values are read only by the other colour: in place (red-black)
            if (MODE != 2)
#pragma unroll
                for (int c = 0; c < 3; ++c) X[c][j] = r[k][c];
        }
        if (MODE == 2) {   // Jacobi: every read of the old iterate before any write
            __syncthreads();
#pragma unroll
            for (int k = 0; k < PER; ++k)
                if (on[k])
#pragma unroll
                    for (int c = 0; c < 3; ++c) X[c][t + NT * k] = r[k][c];
        }
        __syncthreads();
    };
    if constexpr (RB) {
        pass(std::integral_constant<int, 0>{});
        pass(std::integral_constant<int, 1>{});
    } else {
        pass(std::integral_constant<int, 2>{});
    }
#pragma unroll
    for (int k = 0; k < PER; ++k) {   // tnew_nonlin (store 2: tnew)
        const int j = t + NT * k;
        const int64_t s = s0 + j;
        if (s < N)
#pragma unroll
            for (int c = 0; c < 3; ++c) (store == 2 ? T : TNN)[c * pitch + s] = X[c][j];
    }
    if (!next_halo) return;
#pragma unroll
    for (int k = 0; k < PER / 2; ++k) {   // the next sweep's halo words, an adjacent pair per thread
        const int j = 2 * (t + NT * k);
        const int64_t s = s0 + j;
        if (s >= N) continue;
        HaloPre hp;
        halo_prefetch(Hn, s, s >> nsub_log2, nsub_log2, hp);
        const double p0[3] = {X[0][j], X[1][j], X[2][j]}, p1[3] = {X[0][j + 1], X[1][j + 1], X[2][j + 1]};
        halo_write(Hn, hp, p0, p1);
    }
}

// ---- the persistent chain: every sweep of one smoother call in ONE launch, for a level whose
// iterate fits in the LDS of one workgroup per CU (the coarsest level of the face-coupled V-cycle:
// 524,288 sub-elements at n_split = 5, L = 3 -- 62 of the cycle's 74 sweeps). Workgroup w keeps the
// iterate of its un_eles [w k, (w+1) k) in LDS for the whole call (no HBM traffic between sweeps)
// and the RHS in registers. A sweep reads a halo snapshot that the PREVIOUS sweep of every
// neighbouring workgroup wrote (update_overlaps, :555), so the workgroups hand the words over inside
// the launch (cdna_hip_programming.md 6 Guideline 16, R1 with one workgroup per CU): each writes its
// next-sweep words through to the coherent level (st_coh), drains them (s_waitcnt vmcnt(0) in every
// wave, then the barrier) and publishes one flag word, flags[w] = sweeps done; before its sweep s a
// workgroup polls (one wave, relaxed agent-scope loads, s_sleep) the flags of the workgroups owning
// its un_eles' neighbours until each is >= s, and reads the words with ld_coh only. The snapshot
// buffers alternate as in face_call; a neighbour can overwrite buffer (s+1) & 1 only after it has
// seen flags[w] >= s, i.e. after w has finished sweep s - 1, the last reader of that buffer. Every
// sub-element's arithmetic is face_point's, so the result is bitwise the per-sweep launches'. The
// spin is bounded: a workgroup that waits > 2^22 polls sets *tmo and goes on (the host reports the
// call as failed). Resident by construction: grid <= CUs, 1,024 threads, launched cooperatively.
constexpr int kChainNT = 1024, kChainPer = 2;   // threads, sub-elements per thread (<= 2,048 per workgroup)
constexpr int kChainHalo = 9216;                 // LDS image of the halo snapshot (doubles): 9 k m <= 9 * 1024

// the next sweep's halo words of one sub-element (update_overlaps, :555) from its iterate t: h = its
// positions along faces 1..3, 10 bits each, rec the un_ele's face records; bc: also the boundary
// words (constant within a time step: the call's halo refresh writes them into one snapshot buffer,
// the call's first sweep into the other). COH: written through (st_coh) for readers in other
// workgroups of the same launch. The t_overlap_old words (told, constant within a time step) are the
// call's halo refresh's (launch_face_halo), so the sweeps leave them alone.
template <bool COH>
__device__ __forceinline__ void halo_words(const HaloArgs &H, const int4 rec[3], int h, const double t[3], bool bc) {
    const int pos[3] = {h & 1023, (h >> 10) & 1023, h >> 20};
#pragma unroll
    for (int f = 0; f < 3; ++f) {
        const int i = pos[f];
        if (!i) continue;
        const int4 r = rec[f];
        const int mode = r.x & 3;
        if (mode == 0) {
            if (!bc) continue;
            const int a = (i - 1) * 3 + (f == 2 ? 1 : 0);
            const int b = (i - 1) * 3 + (f == 1 ? 1 : 2);
            const double2 v = H.bcv[r.z + i - 1];
            st_halo<COH>(H.tov + r.y + a, v.x);
            st_halo<COH>(H.tov + r.y + b, v.y);
        } else if (mode == 1) {
            const int k = (r.x >> 2) ? (H.m - i + 1) : i;
            double *d = H.tov + r.y + (int64_t)(k - 1) * 3;
#pragma unroll
            for (int c = 0; c < 3; ++c) st_halo<COH>(d + c, t[c]);
        } else {
            double *o = H.send + 6 * (int64_t)(r.z + i - 1);
#pragma unroll
            for (int c = 0; c < 3; ++c) st_halo<COH>(o + c, t[c]);
        }
    }
}

// A thread's sub-elements in the passes ("items", fixed for the whole call): red-black runs each
// colour over its own position list (Level::cpos), so every lane of a pass has a sub-element of that
// colour (one launch per sweep masked half the lanes of each colour pass: twice the fp64 issue);
// Jacobi takes the positions in order. j = storage position in the tile, -1 none; nb its fnb entry,
// b its RHS.
template <int K>
struct Items {
    int j[K];
    int4 nb[K];
    double b[K][3];
};

// one pass (MODE 0 / 1 a colour, 2 Jacobi) of a tile's items (j: tile positions); rec(j, nb, f) calls
// f with the item's un_ele record, un_ele, omega / D row and the un_ele's first tile position; xin reads
// the tile; the rest as face_apply. out(k, r): the item's result --
// stored in place at once by a colour pass (a colour reads only the other colour), held by Jacobi
template <int MODE, int K, class XIN, class HV, class REC, class OUT>
__device__ __forceinline__ void items_pass(const Items<K> &I, const XIN &xin, const HV &hv, const REC &rec, int level1,
                                           double rdt, const OUT &out, int kb = 0, int ke = K) {
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const int j = I.j[k];
        if (j < 0 || k < kb || k >= ke) continue;
        double x[3], r[3];
#pragma unroll
        for (int c = 0; c < 3; ++c) x[c] = xin(c, j);
        rec(j, I.nb[k], [&](const FaceRec &R, int64_t u, const double *wd, int jb) {
            auto xb = [&](int c, int q) { return xin(c, jb + q); };   // un_ele-relative neighbour positions
            face_apply<MODE>(R, xb, x, I.b[k], I.nb[k], u, hv, [&](int i) { return wd[i]; }, level1, rdt, r);
        });
        out(k, r);
        asm volatile("" ::: "memory");   // one item at a time: its record's registers are not held across items
    }
}

template <int TS, int NT, bool RB>
struct WaveShape {
    static constexpr int M = TS == 256 ? 16 : TS == 1024 ? 32 : 64;
    static constexpr int NUP = M * (M + 1) / 2, NDN = M * (M - 1) / 2;   // up / down sub-elements
    static constexpr int KU = RB ? (NUP + NT - 1) / NT : TS / NT, KD = RB ? (NDN + NT - 1) / NT : 1;
};

// ---- one sweep on a tile that is exactly one un_ele (nsub = TS: levels of 256, 1,024 or 4,096
// sub-elements per un_ele): k_face_sweep's sweep with every input the passes read issued at the
// start, side by side with the iterate's and RHS's streams -- the un_ele's operator record (scalar
// registers), its omega / D table and its halo snapshot (LDS), the face positions of the thread's
// halo pairs -- so a tile waits on memory once (k_face_sweep waited on the record, the selector and
// the snapshot word in turn inside each colour pass, then on the halo metadata: SQ 79 % of the waves'
// cycles waiting, r03_b_face_sq.txt). The next sweep's halo words are halo_words' (no told reads).
// Same face_apply arithmetic per sub-element: bitwise k_face_sweep's. (Colour item lists, as in the
// chain, made this HBM-bound sweep slower: 0.91 -> 0.98-1.00 ms of level-1 sweeps per cycle with the
// RHS gathered by colour position from memory or through LDS, profiles/r03_f_face_forms.txt.)
template <int TS, int NT, bool RB>
__global__ __launch_bounds__(NT, (RB && TS <= 1024) ? PAMG_FACE_WAVES : 1) void k_face_tile(
    double *T, double *TNN, const double *SRC, const double *__restrict__ RHS, const double *__restrict__ stc,
    const int4 *__restrict__ fnb, const double *__restrict__ fface, const int *__restrict__ fsx,
    const double *__restrict__ tin, HaloArgs Hn, int next_halo, int bc, int store, int64_t pitch, int slots,
    int level1, double rdt, double *RESout) {
    constexpr int PER = TS / NT, M = TS == 256 ? 16 : TS == 1024 ? 32 : 64, NH = 9 * M;
    static_assert(PER % 2 == 0 && M * M == TS, "whole un_ele tiles, adjacent pairs per thread");
    __shared__ double X[3][TS];
    __shared__ double HI[NH];
    __shared__ double WD[24];
    const int t = threadIdx.x;
    const int64_t u = blockIdx.x, s0 = u * TS;
    int4 nbr[PER];
    double b[PER][3];
    int hp[PER];
    int4 hf[3];
    if (next_halo) {
#pragma unroll
        for (int q = 0; q < PER; ++q) {   // pair k = q / 2: sub-elements 2 (t + NT k) + (q & 1)
            const int4 e = Hn.hsub[2 * (t + NT * (q / 2)) + (q & 1)];
            hp[q] = e.x | (e.y << 10) | (e.z << 20);
        }
#pragma unroll
        for (int f = 0; f < 3; ++f) hf[f] = Hn.hface[3 * u + f];
    }
    FaceRec R;
    load_face_rec(stc, fface, fsx, u, R);
    for (int i = t; i < NH; i += NT) HI[i] = tin[u * slots * 3 + (int64_t)(i / (3 * M)) * slots + i % (3 * M)];
    if (t < 24) WD[t] = fface[u * kFaceStride + kFaceWD + t];
#pragma unroll
    for (int k = 0; k < PER; k += 2) {   // tnew := tnew_nonlin (:550); the iterate into LDS, pairs
        const int j = 2 * (t + NT * (k / 2));
        nbr[k] = fnb[j];
        nbr[k + 1] = fnb[j + 1];
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            const double2 v = ld2(SRC + c * pitch + s0 + j), r = ld2(RHS + c * pitch + s0 + j);
            b[k][c] = r.x;
            b[k + 1][c] = r.y;
            X[c][j] = v.x;
            X[c][j + 1] = v.y;
            if (store == 1 && SRC != T) st2(T + c * pitch + s0 + j, v);
        }
    }
    __syncthreads();
    auto xin = [&](int c, int q) { return X[c][q]; };
    auto hv = [&](int64_t, int mf, int sp, int kk) { return HI[((mf - 1) * M + sp - 1) * 3 + kk]; };
    if (RESout) {   // get_residual (A x - RHS) of the iterate and snapshot the sweep starts from (:555, :869)
#pragma unroll
        for (int k = 0; k < PER; ++k) {
            const int j = 2 * (t + NT * (k / 2)) + (k & 1);   // adjacent pairs (16-B accesses)
            double x[3], r[3];
#pragma unroll
            for (int c = 0; c < 3; ++c) x[c] = X[c][j];
            face_apply<3>(R, xin, x, b[k], nbr[k], u, hv, [&](int) { return 0.0; }, level1, rdt, r);
#pragma unroll
            for (int c = 0; c < 3; ++c) RESout[c * pitch + s0 + j] = r[c];
        }
        __syncthreads();   // every read of the start iterate before the passes rewrite it
    }
    auto pass = [&](auto mc) {
        constexpr int MODE = decltype(mc)::value;
        double r[PER][3];
        bool on[PER];
#pragma unroll
        for (int k = 0; k < PER; ++k) {
            const int j = 2 * (t + NT * (k / 2)) + (k & 1);   // adjacent pairs (16-B accesses)
            const int4 nb = nbr[k];
            on[k] = !((MODE == 0 && !nb.w) || (MODE == 1 && nb.w));
            if (!on[k]) continue;
            double x[3];
#pragma unroll
            for (int c = 0; c < 3; ++c) x[c] = X[c][j];
            const int wb = 3 * face_pattern(nb);
            face_apply<MODE>(R, xin, x, b[k], nb, u, hv, [&](int i) { return WD[wb + i]; }, level1, rdt, r[k]);
            if (MODE != 2)
#pragma unroll
                for (int c = 0; c < 3; ++c) X[c][j] = r[k][c];
        }
        if (MODE == 2) {
            __syncthreads();
#pragma unroll
            for (int k = 0; k < PER; ++k)
                if (on[k])
#pragma unroll
                    for (int c = 0; c < 3; ++c) X[c][2 * (t + NT * (k / 2)) + (k & 1)] = r[k][c];
        }
        __syncthreads();
    };
    if constexpr (RB) {
        pass(std::integral_constant<int, 0>{});
        pass(std::integral_constant<int, 1>{});
    } else {
        pass(std::integral_constant<int, 2>{});
    }
#pragma unroll
    for (int k = 0; k < PER; k += 2) {   // tnew_nonlin (store 2: tnew), pairs
        const int j = 2 * (t + NT * (k / 2));
#pragma unroll
        for (int c = 0; c < 3; ++c) st2((store == 2 ? T : TNN) + c * pitch + s0 + j, make_double2(X[c][j], X[c][j + 1]));
    }
    if (!next_halo) return;
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        if (!hp[q]) continue;
        const int j = 2 * (t + NT * (q / 2)) + (q & 1);
        const double tv[3] = {X[0][j], X[1][j], X[2][j]};
        halo_words<false>(Hn, hf, hp[q], tv, bc != 0);
    }
}

// ---- two sweeps per HBM pass (temporal blocking) of a level whose tile is one un_ele (k_face_tile's
// levels of 256 and 1,024 sub-elements; single domain). Every sweep reads its cross-un_ele values from
// a snapshot of the neighbours' iterate at the sweep's start (:555, Jacobi across un_ele faces, red-black
// or Jacobi inside). Here the snapshot is not published through t_overlap: the launch reads its input
// iterate A (written by the previous launch, read-only in this one -- its output goes to another buffer)
// and takes the neighbours' boundary values straight from it. For a second sweep in the same launch the
// tile needs the neighbours' boundary values after the FIRST sweep -- which their own workgroups are
// computing -- so it computes them itself: every sub-element with halo words is an up one (words_up), an
// up sub-element's sweep reads only its down neighbours (unchanged since the previous sweep) and the
// snapshot across its un_ele faces, so the neighbour v's boundary sub-element e after the sweep is
// face_apply of e's value, its two down neighbours, its RHS and v's operator record -- all in A or in
// memory that does not change -- and the snapshot values across e's faces: this tile's own boundary
// values at the sweep's start, or (corners) those of v's other neighbour w, in A. The same face_apply on
// the same operands as v's own workgroup: bitwise the per-sweep launches (tests/test_face_operator.py).
// A pass: K = 1 or 2 sweeps; res 1: get_residual of the start iterate, 2: of the iterate after the first
// sweep (the residual point of a smoother stream, with the snapshot the second sweep reads); outputs:
// out_pre the start iterate, out_mid the iterate after sweep 1 (K = 2), out_end (and out_end2) the iterate after the
// last sweep (none of them aliases A).
// gtab (U x 3 x m, Level::gtab): the gather entry of every halo slot (see the prologue).
#ifndef PAMG_FACE_PP_WAVES
#define PAMG_FACE_PP_WAVES 6
#endif
// the 256-sub-element instance (level 2 at n_split 5): at six waves per SIMD its two-sweep form spilled
// 84 B per lane; four keep it in 104 VGPRs
#ifndef PAMG_FACE_PP_WAVES256
#define PAMG_FACE_PP_WAVES256 4
#endif
// ... its instances without the folded interpolation (A/B)
#ifndef PAMG_FACE_PP_WAVES256_PLAIN
#define PAMG_FACE_PP_WAVES256_PLAIN 4
#endif
// NT: red-black passes with fewer threads than up sub-elements run a second up item on some threads. For
// the 256-sub-element un_ele 192 threads (136 ups, one each) measured faster than 128 (0.71 vs 0.73 ms of
// coarse launches per cycle); for the 1,024 one 576 threads (528 ups) measured slower than 512 (level-1
// passes 0.85 vs 0.71 ms per cycle at seven waves per SIMD, profiles/r04_k_face_pp_nt.txt), so it keeps 512
// phase stamps of the two-sweep passes (diagnostics build: make PAMG_STAMPS=1 and PAMG_PP_STAMPS=<file>;
// scripts/pp_stamps.py): per workgroup the wall clock (100 MHz) at its start, after its loads, after the ghost
// update, after each sweep and after its stores
constexpr int kPPStamps = 6;
__device__ long long *g_pp_stamps = nullptr;
__device__ __forceinline__ void pp_stamp(int i) {
    if (PAMG_STAMPS && g_pp_stamps && threadIdx.x == 0) g_pp_stamps[(int64_t)blockIdx.x * kPPStamps + i] = wall_clock64();
}

// FOLD: the instance that folds the corrected cycle's interpolation (Tc) or a coarse level's zero start (A null) into
// its loads -- a template parameter, so that the passes without either keep their registers (the folded loads
// spilled 52 B per lane in the level-1 two-sweep instance)
#ifndef PAMG_FACE_PP_FOLD_WAVES
#define PAMG_FACE_PP_FOLD_WAVES PAMG_FACE_PP_WAVES
#endif
// XCD-grouped tiles: blocks b and b + 8 are dealt to one XCD (round-robin, MI355X_MICROARCH.md "Workgroup
// dispatch"; speed only, never correctness), so the tiles are renumbered for the passes to give each XCD a
// contiguous range of un_eles: XCD class x = b % 8 takes [x q + min(x, r), ...) of the G = 8 q + r tiles, in order.
// A tile gathers its neighbours' boundary values (the ghost update's operands, scattered 8-byte loads); with
// neighbours in one contiguous range they are mostly tiles of the same XCD, loaded at about the same time, so the
// gathers hit that XCD's L2 instead of the fabric. A bijection on [0, G).
#ifndef PAMG_FACE_PP_XCD
#define PAMG_FACE_PP_XCD 1
#endif
__device__ __forceinline__ int64_t xcd_tile(unsigned b, unsigned G) {
    const unsigned q = G >> 3, r = G & 7, x = b & 7, i = b >> 3;
    return (int64_t)x * q + (x < r ? x : r) + i;
}

template <int TS, int NT, bool RB, int K, bool FOLD = false>
__global__ __launch_bounds__(NT, RB ? (TS <= 256 ? (FOLD ? PAMG_FACE_PP_WAVES256 : PAMG_FACE_PP_WAVES256_PLAIN) : FOLD ? PAMG_FACE_PP_FOLD_WAVES : PAMG_FACE_PP_WAVES) : 1) void k_face_pp(
    const double *__restrict__ A, double *out_pre, double *out_mid, double *out_end, double *out_end2,
    const double *__restrict__ RHS,
    const double *__restrict__ stc, const int4 *__restrict__ fnb, const double *__restrict__ fface,
    const int *__restrict__ fsx, const int4 *__restrict__ gtab, const int *__restrict__ gpat, const int4 *__restrict__ hface,
    const double2 *__restrict__ bcv, const int *__restrict__ cpos, const int4 *__restrict__ cnb, int nup, int64_t pitch,
    int level1, double rdt,
    int res, double *RESout, double *RHSc, int64_t pitch_c, const double *__restrict__ Tc) {
    constexpr int PER = TS / NT, M = TS == 256 ? 16 : TS == 1024 ? 32 : 64, NH = 9 * M;
    // red-black: the colour passes run over colour lists (Level::cpos), every lane with an item of the colour
    constexpr int NUP = M * (M + 1) / 2, KU = RB ? (NUP + NT - 1) / NT : PER, KD = RB ? (TS - NUP + NT - 1) / NT : 0;
    static_assert((RB || (TS % NT == 0 && PER % 2 == 0)) && M * M == TS && 3 * M <= NT && TS <= 1024,
                  "whole un_ele tiles of <= 1,024; Jacobi: adjacent pairs per thread");
    // one LDS array: the iterate, the RHS, ONE halo snapshot image, omega / D. The second sweep's snapshot -- the
    // ghost updates -- stays in the registers of the threads that compute it and replaces the first sweep's once
    // that sweep's last reader has passed: the up pass (a down sub-element never reads the snapshot, words_up) or
    // Jacobi's read phase. 53,952 -> 51,648 B of LDS: three workgroups per CU instead of two (phase stamps,
    // profiles/r05_n_pp_stamps.txt: 512 of the 768 slots were ever resident). (Measured, not kept: the RHS in
    // registers instead of LDS; the ghost update's operands from LDS after the tile's barrier.)
    constexpr int OX = 0, OB = 3 * TS, OH = 6 * TS, OW = OH + NH;
    __shared__ double LDSM[OW + 24];
    double (*X)[TS] = reinterpret_cast<double (*)[TS]>(LDSM + OX);
    double (*B)[TS] = reinterpret_cast<double (*)[TS]>(LDSM + OB);
    double *WD = LDSM + OW;
    double *const HS = LDSM + OH;   // the snapshot image
    const int t = threadIdx.x;
    // (Measured, not kept: starting the first round's k-th workgroup of a CU k x 4 / 8 / 12 us late, so that the
    // co-resident workgroups' load, sweep and store phases fall apart -- the level-1 passes 0.74 -> 0.75 / 0.76 /
    // 0.80 ms per cycle, profiles/r05_f_face_pp_stagger.txt; a persistent grid looping over tiles spilled 272 B
    // per lane.) The tile body is a lambda called once: 76 -> 70 VGPRs.
    auto tile = [&](const int64_t u) {
    pp_stamp(0);
    const int64_t s0 = u * TS;
    FaceRec R;
    load_face_rec(stc, fface, fsx, u, R);
    if (t < 24) WD[t] = fface[u * kFaceStride + kFaceWD + t];
    // the boundary words of a domain-boundary face mf (1..3) at bcv index bci: update_overlaps' boundary values
    // at the two face nodes (halo_words' placement; the third word is never read)
    auto bcpair = [&](int bci, int mf, int kk) -> double {
        const double2 v = bcv[bci];
        return kk == (mf == 3 ? 1 : 0) ? v.x : kk == (mf == 2 ? 1 : 2) ? v.y : 0.0;
    };
    // halo slot (fu, spu) of this tile: thread t -- a face per wave where the workgroup has three waves or
    // more (the neighbour's operator record then comes through the scalar unit), else packed. Its gather
    // entry (Level::gtab) names, for the neighbour's boundary sub-element e facing the slot, e's global
    // index and, per face of e, the global index of the value across it (>= 0), this tile's own position
    // p as -1 - p, or a boundary word as -(1 + TS + 3 bcv index + face - 1): every operand load of the
    // ghost update below is issued here, at the launch's start, beside the tile's own loads
    constexpr bool WAVEF = NT >= 192;
    const int fu = WAVEF ? t / 64 + 1 : t / M + 1;
    const int spu = WAVEF ? (t & 63) + 1 : t - (fu - 1) * M + 1;
    const bool gon = fu <= 3 && spu <= M;
    const int hq = 3 * ((fu - 1) * M + spu - 1);   // the slot's first word in a snapshot
    int4 ge = make_int4(-1, -1, -1, -1);
    int gp = 0;   // e's face pattern (Level::gpat), loaded beside the entry
    if (gon) {
#if PAMG_DIAG_NOGATHER   // timing diagnostic only (wrong results): no gather entry, no neighbour values, no ghost update
        ge = make_int4(-3, 0, 0, 0);
#else
        ge = gtab[(u * 3 + fu - 1) * M + spu - 1];
        gp = gpat[(u * 3 + fu - 1) * M + spu - 1];
#endif
    }
    // the start iterate at global position g: A's value, plus the prolonged coarse correction where Tc is given (the
    // corrected cycle's interp_add, k_interp_add's arithmetic, folded into the first pass of the smoother call that
    // follows it), or zero where A is null (a coarse level's call from zero: the cycle's memset folded)
    auto ldv = [&](int64_t g, double v[3]) {
#pragma unroll
        for (int c = 0; c < 3; ++c) v[c] = !FOLD || A ? A[c * pitch + g] : 0.0;
        if (FOLD && Tc) {
            const int64_t cg = g >> 2;
            const double y[3] = {Tc[cg], Tc[pitch_c + cg], Tc[2 * pitch_c + cg]};
            double add[3];
            interp_corr((int)(g & 3), y, add);
#pragma unroll
            for (int c = 0; c < 3; ++c) v[c] = v[c] + add[c];
        }
    };
    double xe[3] = {0.0, 0.0, 0.0}, be[3] = {0.0, 0.0, 0.0}, yv[3][3];
    int4 nbe = make_int4(0, 0, 0, 0);
    if (gon && ge.x >= 0) {
        // fnb[e]'s signs, all face_core and face_pattern read of it
        nbe = make_int4((gp & 1) ? 0 : -1, (gp & 2) ? 0 : -1, (gp & 4) ? 0 : -1, 0);
        ldv(ge.x, xe);
        if (K == 2)
#pragma unroll
            for (int c = 0; c < 3; ++c) be[c] = RHS[c * pitch + ge.x];
        if constexpr (K == 2) {
            const int yy[3] = {ge.y, ge.z, ge.w};
#pragma unroll
            for (int fi = 0; fi < 3; ++fi) {
                if (yy[fi] >= 0) {
                    ldv(yy[fi], yv[fi]);
                } else if (yy[fi] > -(1 + TS)) {
                    ldv(s0 - 1 - yy[fi], yv[fi]);   // this tile's own start value, as its bulk load forms it
                } else {
#pragma unroll
                    for (int c = 0; c < 3; ++c)
                        yv[fi][c] = yy[fi] <= -(1 + TS) ? bcpair((-(yy[fi] + 1 + TS)) / 3, (-(yy[fi] + 1 + TS)) % 3 + 1, c)
                                                        : 0.0;   // this tile's own value: from LDS below
                }
            }
        }
    }
    // the thread's items: red-black -- KU up and KD down positions from the colour lists; Jacobi -- its PER
    // positions (adjacent pairs)
    int ij[KU + KD];
    int4 inb[KU + KD];
#pragma unroll
    for (int k = 0; k < KU + KD; ++k) {
        if constexpr (RB) {
            const int i = k < KU ? t + NT * k : NUP + t + NT * (k - KU);
            const bool in = k < KU ? i < NUP : i < TS;
            ij[k] = in ? cpos[i] : -1;
            inb[k] = cnb[in ? i : 0];   // fnb[cpos[i]], loaded beside cpos[i]
        } else {
            ij[k] = 2 * (t + NT * (k / 2)) + (k & 1);
            inb[k] = fnb[ij[k]];
        }
    }
    (void)nup;
    // unless the start iterate is stored (out_pre), the RHS -- and the start iterate when it is read
    // (not a start from zero) -- go to LDS by LDS-DMA: a wave's 64 pairs of a plane are one 1 KiB global_load_lds_dwordx4
    // into X / B (lane-linear), no VGPR round trip; in the folded instance an interpolation is then added to X in place
    // by the pair's own thread (after its wave's wait: its lane wrote that pair), v + a as in the register path; the
    // __syncthreads below waits for the rest
    const bool gr = !out_pre, ga = gr && (!FOLD || A);
    if (gr) {
        constexpr int aux = (PAMG_NT & 1) ? 2 : 0;
        const int lane = t & 63;
        for (int p0 = t - lane; p0 < TS / 2; p0 += NT) {   // wave-uniform: the wave's first pair
            const int j0 = 2 * p0;
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                if (ga)
                    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)(A + c * pitch + s0 + j0 + 2 * lane),
                                                     (__attribute__((address_space(3))) void *)(&X[c][j0]), 16, 0, aux);
                __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)(RHS + c * pitch + s0 + j0 + 2 * lane),
                                                 (__attribute__((address_space(3))) void *)(&B[c][j0]), 16, 0, aux);
            }
        }
        if (FOLD && ga && Tc) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    if constexpr (!FOLD) {
#pragma unroll
        for (int p = gr ? TS : t; p < TS / 2; p += NT) {   // the iterate and the RHS into LDS, adjacent pairs
            const int j = 2 * p;
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                const double2 v = ld2(A + c * pitch + s0 + j);
                const double2 r = ld2(RHS + c * pitch + s0 + j);
                X[c][j] = v.x;
                X[c][j + 1] = v.y;
                B[c][j] = r.x;
                B[c][j + 1] = r.y;
                if (out_pre) st2(out_pre + c * pitch + s0 + j, v);
            }
        }
    } else {
#pragma unroll
        for (int p = ga && !Tc ? TS : t; p < TS / 2; p += NT) {   // the iterate (and the RHS) into LDS, adjacent pairs
            const int j = 2 * p;
            double a0[3] = {0.0, 0.0, 0.0}, a1[3] = {0.0, 0.0, 0.0};
            if (Tc) {   // ldv's correction: both children of the pair share their coarse sub-element
                const int64_t cg = (s0 + j) >> 2;
                const double y[3] = {Tc[cg], Tc[pitch_c + cg], Tc[2 * pitch_c + cg]};
                interp_corr(j & 3, y, a0);
                interp_corr((j + 1) & 3, y, a1);
            }
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                double2 v;
                if (ga) v = make_double2(X[c][j], X[c][j + 1]);   // Tc: the DMA's value
                else v = A ? ld2(A + c * pitch + s0 + j) : make_double2(0.0, 0.0);
                if (Tc) v = make_double2(v.x + a0[c], v.y + a1[c]);
                X[c][j] = v.x;
                X[c][j + 1] = v.y;
                if (!gr) {
                    const double2 r = ld2(RHS + c * pitch + s0 + j);
                    B[c][j] = r.x;
                    B[c][j + 1] = r.y;
                }
                if (out_pre) st2(out_pre + c * pitch + s0 + j, v);
            }
        }
    }
    // the snapshot of the first sweep (:555 at its start): the neighbours' boundary values in A, or this
    // tile's boundary words
    if (gon)
#pragma unroll
        for (int kk = 0; kk < 3; ++kk)
            HS[hq + kk] = ge.x >= 0 ? xe[kk] : ge.x == -1 ? bcpair(hface[3 * u + fu - 1].z + spu - 1, fu, kk) : 0.0;
    // the neighbour's operator record for the ghost update (scalar loads, in flight across the barrier)
    FaceRec Rv;
    const double *wdv = nullptr;
    if (K == 2 && gon && ge.x >= 0) {
        const int64_t v = WAVEF ? __builtin_amdgcn_readfirstlane(ge.x / TS) : ge.x / TS;   // one face a wave
        load_face_rec(stc, fface, fsx, v, Rv);
        wdv = fface + v * kFaceStride + kFaceWD + 3 * face_pattern(nbe);
    }
    double hn[3] = {0.0, 0.0, 0.0};   // this thread's slot of the second sweep's snapshot
    // the neighbour's boundary sub-element e after the first sweep (an up one: its sweep reads its down
    // neighbours, unchanged since the previous sweep, and the snapshot across its faces): the second
    // sweep's snapshot -- face_core on v's record and the values gathered above. Every operand came from
    // memory, so the update runs as soon as they arrive, before the tile's barrier (no LDS read, no second barrier)
    auto ghost = [&]() {
        if (gon) {
            if (ge.x >= 0) {
                double r[3];
                // (the component of a halo word is a run-time selector: picked by selects, so that yv stays in
                // registers)
                face_core<RB ? 0 : 2>(Rv, xe, be, nbe,
                                      [&](int fi, int c) { return c == 0 ? yv[fi][0] : c == 1 ? yv[fi][1] : yv[fi][2]; },
                                      [&](int q) { return wdv[q]; }, level1, rdt, r);
#pragma unroll
                for (int c = 0; c < 3; ++c) hn[c] = r[c];
            }
        }
    };
    if constexpr (K == 2) ghost();
    __syncthreads();
    pp_stamp(1);
    if constexpr (K == 2) pp_stamp(2);
    // the second sweep's snapshot into the image, after the first sweep's last read of it (boundary words: constant)
    auto snap_next = [&]() {
        if (K == 2 && gon && ge.x >= 0)
#pragma unroll
            for (int c = 0; c < 3; ++c) HS[hq + c] = hn[c];
    };
    auto xin = [&](int c, int q) { return X[c][q]; };
    // one item k: face_apply<MODE> of position ij[k] from the tile, the RHS and snapshot snap
    auto item = [&](auto mc, int k, int snap, double r[3]) {
        constexpr int MODE = decltype(mc)::value;
        const int j = ij[k];
        const double *H = HS;
        (void)snap;
        auto hv = [&](int64_t, int mf, int sp, int kk) { return H[((mf - 1) * M + sp - 1) * 3 + kk]; };
        double x[3], bb[3];
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            x[c] = X[c][j];
            bb[c] = B[c][j];
        }
        const int wb = 3 * face_pattern(inb[k]);
        face_apply<MODE>(R, xin, x, bb, inb[k], u, hv, [&](int i) { return MODE == 3 ? 0.0 : WD[wb + i]; }, level1, rdt, r);
    };
    // get_residual of the tile's iterate with snapshot snap: MODE 3 A x - RHS (res 1 / 2, the reference cycle's), 4
    // RHS - A x (res 3, the corrected cycle's). Stored into RESout where given; restricted into RHSc where given
    // (k_restrict_tile's restrictor: the coarse sub-element cc of this tile takes component i from child pick_i =
    // 4 cc + {2, 3, 0}[i], the mean of that child's three residual components, in k_restrict_tile's order -- so
    // each item writes its coarse value itself, and child 4 cc + 1 is not evaluated unless RESout is stored)
    auto residual = [&](auto mc, int snap) {
        const int64_t c0 = s0 >> 2;
#pragma unroll
        for (int k = 0; k < KU + KD; ++k) {
            const int j = ij[k];
            if (j < 0 || (!RESout && (j & 3) == 1)) continue;
            double r[3];
            item(mc, k, snap, r);
            if (RESout)
#pragma unroll
                for (int c = 0; c < 3; ++c) RESout[c * pitch + s0 + j] = r[c];
            const int q = j & 3;
            if (RHSc && q != 1) RHSc[(q == 2 ? 0 : q == 3 ? 1 : 2) * pitch_c + c0 + (j >> 2)] = div3(r[0] + r[1] + r[2]);
        }
    };
    auto sweep = [&](int snap) {
        if constexpr (RB) {   // up items, then down items, in place (a colour reads only the other)
#pragma unroll
            for (int k = 0; k < KU; ++k) {
                if (ij[k] < 0) continue;
                double r[3];
                item(std::integral_constant<int, 0>{}, k, snap, r);
#pragma unroll
                for (int c = 0; c < 3; ++c) X[c][ij[k]] = r[c];
            }
            __syncthreads();
            if (snap == 0) snap_next();   // the down pass reads no snapshot
#pragma unroll
            for (int k = KU; k < KU + KD; ++k) {
                if (ij[k] < 0) continue;
                double r[3];
                item(std::integral_constant<int, 1>{}, k, snap, r);
#pragma unroll
                for (int c = 0; c < 3; ++c) X[c][ij[k]] = r[c];
            }
            __syncthreads();
        } else {   // Jacobi: every read of the old iterate before any write
            double r[KU][3];
#pragma unroll
            for (int k = 0; k < KU; ++k) item(std::integral_constant<int, 2>{}, k, snap, r[k]);
            __syncthreads();
            if (snap == 0) snap_next();
#pragma unroll
            for (int k = 0; k < KU; ++k)
#pragma unroll
                for (int c = 0; c < 3; ++c) X[c][ij[k]] = r[k][c];
            __syncthreads();
        }
    };
    auto store = [&](double *o) {
#pragma unroll
        for (int p = t; p < TS / 2; p += NT) {
            const int j = 2 * p;
#pragma unroll
            for (int c = 0; c < 3; ++c) st2(o + c * pitch + s0 + j, make_double2(X[c][j], X[c][j + 1]));
        }
    };
    if (res == 3) {   // the corrected cycle's get_residual and restrictor (:336-338): no sweep, no stores of the iterate
        residual(std::integral_constant<int, 4>{}, 0);
        return;
    }
    if (res == 1) {
        residual(std::integral_constant<int, 3>{}, 0);
        __syncthreads();   // every read of the iterate before the passes rewrite it
    }
    sweep(0);
    pp_stamp(3);
    if constexpr (K == 2) {
        if (out_mid) store(out_mid);
        if (res == 2) {
            residual(std::integral_constant<int, 3>{}, 1);
            __syncthreads();
        }
        sweep(1);
    }
    pp_stamp(4);
    if (out_end) store(out_end);
    if (out_end2) store(out_end2);   // the corrected cycle's smoother call: tnew and tnew_nonlin both its result
    if (PAMG_STAMPS) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    pp_stamp(5);
    };
    tile(PAMG_FACE_PP_XCD ? xcd_tile(blockIdx.x, gridDim.x) : (int64_t)blockIdx.x);
}

// ---- the wavefront call: every sweep of one smoother call on a level too large to stay on-chip
// (levels 1 and 2 at n_split = 5: 8.4 M and 2.1 M sub-elements), each un_ele crossing HBM once per
// call instead of once per sweep. A persistent cooperative grid of G workgroups takes un_eles in
// ticket order (`order`: a reverse Cuthill-McKee numbering of the un_ele graph, host-built, band b);
// a workgroup keeps its un_ele's iterate in LDS and its RHS in registers for the whole call and runs
// sweep s once every neighbour has published its words for sweep s (flags[v] >= s, per un_ele), the
// chain's hand-off (write-through halo words, drain, barrier, flag; ld_coh reads; snapshot buffers by
// parity, safe for the chain's reason: a neighbour overwrites the buffer of sweep s - 1 only after
// this un_ele has published sweep s, i.e. after it read that snapshot). Progress: the lowest
// unfinished ticket t0 is resident, tickets [t0, t0 + G) are claimed, and a ticket in
// [t0, t0 + G - k b) can always reach sweep k -- so G >= (run - 1) b + 1 (face_wave_ok) guarantees
// the grid drains; the spins are bounded anyway (*tmo, as the chain). Every sub-element's arithmetic
// is face_apply's on the same snapshot words, so the result is bitwise the per-sweep launches'.
// Tagged halo granules (cdna_hip_programming.md 6 Guideline 16, R2: the data is the flag). A halo
// double d of sweep s travels as two 8-byte words {lo32(d), tag}, {hi32(d), tag}, each one aligned
// agent-scope atomic store (single-copy atomic), tag = the launch's tag base + s. A reader re-reads
// both words (agent-scope atomic loads) until both carry the tag it expects, then has the exact
// double: no flag, no drain, no fence, any number of workgroups per CU, and a tear between the two
// words is caught by the tags. Granule buffers alternate by sweep parity as the snapshot buffers.
typedef unsigned long long u64_t;
__device__ __forceinline__ void st_gran(u64_t *g, double d, unsigned tag) {
    const u64_t b = (u64_t)__double_as_longlong(d);
    __hip_atomic_store((g_u64 *)g, (b & 0xffffffffull) | ((u64_t)tag << 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store((g_u64 *)(g + 1), (b >> 32) | ((u64_t)tag << 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// poll up to B granules at once (gi[b] < 0: none) into LDS (HI[li[b]]): every pending granule's two
// words are requested together, so a round trip serves all of them; only the ones whose tags did not
// match yet are re-read (bounded: *tmo set after 2^22 rounds)
template <int B>
__device__ __forceinline__ void gran_poll(const u64_t *gin, unsigned tag, const int64_t (&gi)[B], const int (&li)[B],
                                          double *HI, unsigned *tmo) {
    bool need[B];
#pragma unroll
    for (int b = 0; b < B; ++b) need[b] = gi[b] >= 0;
    for (unsigned spins = 0;; ++spins) {
        u64_t x[B], y[B];
#pragma unroll
        for (int b = 0; b < B; ++b)
            if (need[b]) {
                x[b] = __hip_atomic_load((g_u64 *)const_cast<u64_t *>(gin + 2 * gi[b]), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                y[b] = __hip_atomic_load((g_u64 *)const_cast<u64_t *>(gin + 2 * gi[b] + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        bool more = false;
#pragma unroll
        for (int b = 0; b < B; ++b)
            if (need[b]) {
                if ((unsigned)(x[b] >> 32) == tag && (unsigned)(y[b] >> 32) == tag) {
                    HI[li[b]] = __longlong_as_double((long long)((x[b] & 0xffffffffull) | (y[b] << 32)));
                    need[b] = false;
                } else {
                    more = true;
                }
            }
        if (!more) return;
        if (spins > (1u << 22)) {
            __hip_atomic_store((g_u32 *)tmo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            return;
        }
        __builtin_amdgcn_s_sleep(1);
    }
}

// the next sweep's halo words of one sub-element as granules (update_overlaps, :555; halo_words'
// destinations): a neighbour on this rank gets the granules of sweep `tag`, and, when fin, the plain
// t_overlap word as well (the state the call leaves); the domain-boundary words (constant in a time
// step) go plain into the snapshot buffer, at the call's first sweep (bc)
__device__ __forceinline__ void halo_gran(const HaloArgs &H, const int4 rec[3], int h, const double t[3], bool bc,
                                          u64_t *gout, unsigned tag, bool fin) {
    const int pos[3] = {h & 1023, (h >> 10) & 1023, h >> 20};
#pragma unroll
    for (int f = 0; f < 3; ++f) {
        const int i = pos[f];
        if (!i) continue;
        const int4 r = rec[f];
        const int mode = r.x & 3;
        if (mode == 0) {
            if (!bc) continue;
            const int a = (i - 1) * 3 + (f == 2 ? 1 : 0);
            const int b = (i - 1) * 3 + (f == 1 ? 1 : 2);
            const double2 v = H.bcv[r.z + i - 1];
            H.tov[r.y + a] = v.x;
            H.tov[r.y + b] = v.y;
        } else if (mode == 1) {
            const int k = (r.x >> 2) ? (H.m - i + 1) : i;
            const int64_t d = r.y + (int64_t)(k - 1) * 3;
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                if (gout) st_gran(gout + 2 * (d + c), t[c], tag);
                if (fin) H.tov[d + c] = t[c];
            }
        }
    }
}

constexpr int kWaveStampT = 32, kWaveStampW = 19;   // tickets per workgroup, stamps per ticket
#ifndef PAMG_WAVE_WAVES
#define PAMG_WAVE_WAVES 4
#endif

template <int TS, int NT, bool RB>
__global__ __launch_bounds__(NT, TS <= 1024 ? PAMG_WAVE_WAVES : 1) void k_face_wave(
    double *T, double *TNN, const double *SRC, const double *__restrict__ RHS, const double *__restrict__ stc,
    const int4 *__restrict__ fnb, const double *__restrict__ fface, const int *__restrict__ fsx,
    const int *__restrict__ cpos, int nup, double *buf0, double *buf1, u64_t *g0, u64_t *g1, unsigned tag0,
    HaloArgs H, unsigned *flags, const int *__restrict__ order, unsigned *tmo, int U, int run, int total,
    int store, int64_t pitch, int slots, int level1, double rdt, long long *stamps) {
    using WS = WaveShape<TS, NT, RB>;
    constexpr int PER = TS / NT, M = WS::M, NH = 9 * M, KU = WS::KU, KD = WS::KD;
    static_assert(PER % 2 == 0 && M * M == TS, "whole un_ele tiles, adjacent pairs per thread");
    __shared__ double X[3][TS];
    __shared__ double HI[NH];
    __shared__ double WD[24];
    __shared__ int s_tk;
    const int t = threadIdx.x;
    unsigned *ticket = flags + U;   // the claim counter sits after the per-un_ele flags
    int hp[PER];
#pragma unroll
    for (int q = 0; q < PER; ++q) {   // face positions of the thread's halo pairs (the same in every un_ele)
        const int4 e = H.hsub[2 * (t + NT * (q / 2)) + (q & 1)];
        hp[q] = e.x | (e.y << 10) | (e.z << 20);
    }
    // the thread's items: the first colour (all positions for Jacobi), then the second
    Items<KU> IA;
    Items<KD> IB;
#pragma unroll
    for (int k = 0; k < KU; ++k) {
        const int i = t + NT * k;
        IA.j[k] = RB ? (i < nup ? cpos[i] : -1) : i;
        IA.nb[k] = fnb[IA.j[k] < 0 ? 0 : IA.j[k]];
    }
#pragma unroll
    for (int k = 0; k < KD; ++k) {
        const int i = t + NT * k;
        IB.j[k] = RB && i < TS - nup ? cpos[nup + i] : -1;
        IB.nb[k] = fnb[IB.j[k] < 0 ? 0 : IB.j[k]];
    }
    // diagnostics (PAMG_WAVE_STAMPS): per ticket of workgroups 0..7 (the first kWaveStampT), wall
    // clock at the claim, after the state's load, per sweep after the wait / snapshot / passes /
    // publish, at the end
    int nt_w = 0;
    for (;;) {
        if (t == 0) s_tk = (int)__hip_atomic_fetch_add((g_u32 *)ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __syncthreads();
        const int tk = s_tk;
        if (tk >= U) break;
        long long *st = (stamps && t == 0 && blockIdx.x < 8 && nt_w < kWaveStampT)
                            ? stamps + ((int64_t)blockIdx.x * kWaveStampT + nt_w) * kWaveStampW
                            : nullptr;
        ++nt_w;
        if (st) st[0] = wall_clock64();
        const int64_t u = __builtin_amdgcn_readfirstlane(order[tk]);
        const int64_t s0 = u * TS;
        int4 hf[3];
#pragma unroll
        for (int f = 0; f < 3; ++f) hf[f] = H.hface[3 * u + f];
        FaceRec R;
        load_face_rec(stc, fface, fsx, u, R);
        if (t < 24) WD[t] = fface[u * kFaceStride + kFaceWD + t];
#pragma unroll
        for (int k = 0; k < PER; ++k) {
            const int j = t + NT * k;
#pragma unroll
            for (int c = 0; c < 3; ++c) X[c][j] = SRC[c * pitch + s0 + j];
        }
#pragma unroll
        for (int k = 0; k < KU; ++k)
#pragma unroll
            for (int c = 0; c < 3; ++c) IA.b[k][c] = IA.j[k] < 0 ? 0.0 : RHS[c * pitch + s0 + IA.j[k]];
#pragma unroll
        for (int k = 0; k < KD; ++k)
#pragma unroll
            for (int c = 0; c < 3; ++c) IB.b[k][c] = IB.j[k] < 0 ? 0.0 : RHS[c * pitch + s0 + IB.j[k]];
        // which of the un_ele's faces have a neighbour on this rank (their words arrive as granules;
        // a domain-boundary face's words are constant and come with the sweep-0 snapshot)
        const int nbm = ((hf[0].x & 3) == 1) | (((hf[1].x & 3) == 1) << 1) | (((hf[2].x & 3) == 1) << 2);
        if (st) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            st[1] = wall_clock64();
        }
        auto xin = [&](int c, int q) { return X[c][q]; };
        auto hv = [&](int64_t, int mf, int sp, int kk) { return HI[((mf - 1) * M + sp - 1) * 3 + kk]; };
        auto rec = [&](int, int4 nb, auto &&f) { f(R, u, WD + 3 * face_pattern(nb), 0); };
        for (int sw = 0; sw < run; ++sw) {
            const double *tin = ((total - 1 - sw) & 1) ? buf1 : buf0;
            double *tout = sw + 1 < total ? (((total - 2 - sw) & 1) ? buf1 : buf0) : nullptr;
            // the items' positions and neighbour entries re-read in every sweep (small tables, cache
            // hits) behind an opaque index, so that they and the LDS addresses derived from them are
            // not held in registers across the sweep loop (VGPRs: occupancy)
#pragma unroll
            for (int k = 0; k < KU; ++k) {
                int i = t + NT * k;
                asm volatile("" : "+v"(i));
                IA.j[k] = RB ? (i < nup ? cpos[i] : -1) : i;
                IA.nb[k] = fnb[IA.j[k] < 0 ? 0 : IA.j[k]];
            }
#pragma unroll
            for (int k = 0; k < KD; ++k) {
                int i = t + NT * k;
                asm volatile("" : "+v"(i));
                IB.j[k] = RB && i < TS - nup ? cpos[nup + i] : -1;
                IB.nb[k] = fnb[IB.j[k] < 0 ? 0 : IB.j[k]];
            }
            const int sk = 2 + 4 * (sw < 4 ? sw : 3);
            if (st) st[sk] = wall_clock64();
            if (sw == 0) {   // the call's snapshot of sweep 0 (the preceding halo launch wrote it)
                for (int i = t; i < NH; i += NT) HI[i] = tin[u * slots * 3 + (int64_t)(i / (3 * M)) * slots + i % (3 * M)];
            } else {         // the neighbours' granules of sweep sw, polled until every tag matches
                constexpr int QB = (NH + NT - 1) / NT;   // the thread's snapshot words, polled together
                int64_t gi[QB];
                int li[QB];
#pragma unroll
                for (int q = 0; q < QB; ++q) {
                    const int i = t + NT * q, f = i / (3 * M);
                    li[q] = i;
                    gi[q] = i < NH && ((nbm >> f) & 1) ? u * slots * 3 + (int64_t)f * slots + i % (3 * M) : -1;
                }
                gran_poll<QB>((sw & 1) ? g1 : g0, tag0 + (unsigned)sw, gi, li, HI, tmo);
            }
            // the call's last sweep: tnew := tnew_nonlin (:550), before the barrier that lets the passes
            // rewrite X (a position's item may belong to another thread)
            if (store == 1 && sw + 1 == run) {
                int tt = t;   // opaque: the store addresses are not held across the sweep loop
                asm volatile("" : "+v"(tt));
#pragma unroll
                for (int k = 0; k < PER; ++k)
#pragma unroll
                    for (int c = 0; c < 3; ++c) T[c * pitch + s0 + tt + NT * k] = X[c][tt + NT * k];
            }
            __syncthreads();
            if (st) st[sk + 1] = wall_clock64();
            if constexpr (RB) {   // up sub-elements, then down ones, in place (a colour reads only the other)
                items_pass<0>(IA, xin, hv, rec, level1, rdt, [&](int k, const double r[3]) {
#pragma unroll
                    for (int c = 0; c < 3; ++c) X[c][IA.j[k]] = r[c];
                });
                __syncthreads();
                items_pass<1>(IB, xin, hv, rec, level1, rdt, [&](int k, const double r[3]) {
#pragma unroll
                    for (int c = 0; c < 3; ++c) X[c][IB.j[k]] = r[c];
                });
            } else {   // Jacobi: every read of the old iterate before any write
                double rj[KU][3];
                items_pass<2>(IA, xin, hv, rec, level1, rdt, [&](int k, const double r[3]) {
#pragma unroll
                    for (int c = 0; c < 3; ++c) rj[k][c] = r[c];
                });
                __syncthreads();
#pragma unroll
                for (int k = 0; k < KU; ++k)
#pragma unroll
                    for (int c = 0; c < 3; ++c) X[c][IA.j[k]] = rj[k][c];
            }
            __syncthreads();
            if (st) st[sk + 2] = wall_clock64();
            if (tout) {   // the next sweep's halo words (:550, :555 of sweep sw + 1) as granules
                HaloArgs Hn = H;
                Hn.tov = tout;
                u64_t *gout = ((sw + 1) & 1) ? g1 : g0;
                const unsigned tag = tag0 + (unsigned)(sw + 1);
                const bool fin = sw + 2 == total;   // the words t_overlap keeps after the call
                // granules only for a sweep this call runs (a dead last sweep has no reader)
                if (sw + 1 >= run) gout = nullptr;
#pragma unroll
                for (int q = 0; q < PER; ++q) {
                    // opaque per sweep: the destinations are recomputed here instead of hoisted
                    // out of the sweep loop (that held ~80 more VGPRs)
                    int hq = hp[q];
                    asm volatile("" : "+v"(hq));
                    if (!hq) continue;
                    const int j = 2 * (t + NT * (q / 2)) + (q & 1);
                    const double tv[3] = {X[0][j], X[1][j], X[2][j]};
                    halo_gran(Hn, hf, hq, tv, sw == 0, gout, tag, fin);
                }
            }
            if (st) st[sk + 3] = wall_clock64();
        }
#pragma unroll
        for (int k = 0; k < PER; ++k) {   // tnew_nonlin (store 2: tnew, the dead last sweep's :550)
            const int j = t + NT * k;
#pragma unroll
            for (int c = 0; c < 3; ++c) (store == 2 ? T : TNN)[c * pitch + s0 + j] = X[c][j];
        }
        if (st) st[kWaveStampW - 1] = wall_clock64();
        __syncthreads();   // s_tk and X are rewritten by the next ticket
    }
}

// The co-residency guard of a chain launch. A chain's workgroups wait on each other's
// flags, so they must all be resident at once; the launch checks the occupancy bound (launch_coresident),
// but a CU-masked stream, another stream's kernels or another process can still hold CUs. Before touching any
// state every workgroup counts its arrival in g[0]; all proceed once all `grid` have arrived, and if one has
// waited kGuardTicks (200 us) in vain it sets the abort bit in the same word -- by compare-and-swap, only while
// the count is short, so either every workgroup proceeds or none does -- and counts the abort in *aborted.
// Late arrivals see the bit and leave. An aborted launch leaves the state untouched: the host reads *aborted
// and runs the call with one launch per sweep instead (pamg_api.cpp face_call). g[1] counts the workgroups
// leaving; the last one re-zeroes g[0] and g[1] for the next launch (stream order: nothing else runs on them).
constexpr unsigned kGuardAbort = 0x80000000u;
constexpr long long kGuardTicks = 20000;   // wall clock, 100 MHz
__device__ __forceinline__ bool chain_enter(unsigned *g, unsigned *aborted) {
    __shared__ int go;
    if (threadIdx.x == 0) {
        const unsigned grid = gridDim.x;
        unsigned v = __hip_atomic_fetch_add((g_u32 *)g, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1;
        const long long t0 = wall_clock64();
        int r = -1;
        while (r < 0) {
            if (v & kGuardAbort) {
                r = 0;
            } else if ((v & 0xffffu) >= grid) {
                r = 1;
            } else if (wall_clock64() - t0 > kGuardTicks) {
                unsigned want = v;
                if (__hip_atomic_compare_exchange_strong((g_u32 *)g, &want, v | kGuardAbort, __ATOMIC_RELAXED,
                                                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
                    __hip_atomic_fetch_add((g_u32 *)aborted, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    r = 0;
                } else {
                    v = want;   // the word moved: decide on its new value
                }
            } else {
                __builtin_amdgcn_s_sleep(2);
                v = __hip_atomic_load((g_u32 *)g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        go = r;
    }
    __syncthreads();
    return go != 0;
}
// The launch's gate (ChainGate, pamg_internal.h; null gate: the host reads *aborted after the launch): the last
// workgroup out reports the launch in the host's pinned status ring (seq << 1 | aborted) and, when it ran, adds 1 to
// the gate signal the stream waits on before the call's next launch -- an aborted launch leaves the stream waiting
// until the host has run the fallback (pamg_api.cpp face_gates_drain)
__device__ __forceinline__ void chain_leave(unsigned *g, const ChainGate &G) {
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned e = __hip_atomic_fetch_add((g_u32 *)g + 1, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
        if (e + 1 == gridDim.x) {
            const unsigned ab = __hip_atomic_load((g_u32 *)g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & kGuardAbort;
            __hip_atomic_store((g_u32 *)g, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store((g_u32 *)g + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (G.gate) {
                __hip_atomic_store(G.stat + (G.seq & (kGateRing - 1)), (G.seq << 1) | (ab ? 1ull : 0ull), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_SYSTEM);
                if (!ab) __hip_atomic_fetch_add(G.gate, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
        }
    }
}

// LREC: the workgroup's un_eles' operator records (FaceRec + omega / D) sit in LDS for the whole call
// (at most kChainRec un_eles): the passes read them there instead of fetching them from memory in
// every pass (the dependent record fetches were most of a sweep's pass time, r03 stamps)
constexpr int kChainRec = 32, kRecW = 48;
// the records of the workgroup's kv un_eles u0 .. into LDS, kRecW doubles each: S.c, S.K[9], S.w[3], the
// face weights w[6], the omega / D table (24), the un_ele faces' node selectors (3)
__device__ __forceinline__ void chain_load_recs(double *RS, const double *__restrict__ stc, const double *__restrict__ fface,
                                                const int *__restrict__ fsx, int64_t u0, int kv, int t, int nt) {
    for (int i = t; i < kv * kRecW; i += nt) {
        const int uk = i / kRecW, q = i - uk * kRecW;
        const int64_t u = u0 + uk;
        double v = 0.0;
        if (q == 0) v = stc[u * kStcStride + kStcC];
        else if (q < 10) v = stc[u * kStcStride + kStcK + q - 1];
        else if (q < 13) v = stc[u * kStcStride + kStcW + q - 10];
        else if (q < 19) v = fface[u * kFaceStride + q - 13];
        else if (q < 43) v = fface[u * kFaceStride + kFaceWD + q - 19];
        else if (q < 46) v = (double)fsx[4 * u + fmface(q - 43) - 1];
        RS[i] = v;
    }
}
// item j's record from the LDS copy: f(R, un_ele, omega / D row, the un_ele's first tile position)
template <class F>
__device__ __forceinline__ void chain_rec(const double *RS, int j, int4 nb, int nsub_log2, int64_t u0, F &&f) {
    const int uk = j >> nsub_log2;
    const double *rs = RS + uk * kRecW;
    FaceRec R;
    R.S.c = rs[0];
#pragma unroll
    for (int q = 0; q < 9; ++q) R.S.K[q] = rs[1 + q];
#pragma unroll
    for (int q = 0; q < 3; ++q) R.S.w[q] = rs[10 + q];
#pragma unroll
    for (int q = 0; q < 6; ++q) R.w[q] = rs[13 + q];
#pragma unroll
    for (int q = 0; q < 3; ++q) R.sx[q] = (int)rs[43 + q];
    f(R, u0 + uk, rs + 19 + 3 * face_pattern(nb), uk << nsub_log2);
}
typedef unsigned v4u __attribute__((ext_vector_type(4)));
constexpr int kAuxSc1 = 16;   // buffer instruction cache policy: sc1 (through to the coherent level)   // un_eles, doubles per record: S 13 | w 6 | WD 24 | sx 3
template <bool UNI, bool RB, bool LREC>
__global__ __launch_bounds__(kChainNT, 1) void k_face_chain(double *T, double *TNN, const double *SRC, const double *__restrict__ RHS,
                                                          const double *__restrict__ stc, const int4 *__restrict__ fnb,
                                                          const double *__restrict__ fface, const int *__restrict__ fsx,
                                                          double *buf0, double *buf1, HaloArgs H, unsigned *flags,
                                                          const int *__restrict__ nb_off, const int *__restrict__ nb_list,
                                                          unsigned *tmo, int run, int total, int store, int E,
                                                          int64_t pitch, int64_t N, int nsub_log2, int slots, int level1,
                                                          double rdt, double omega, const int *__restrict__ cpos,
                                                          int nup, int nui, int early, unsigned f0, int snap_ok,
                                                          long long *stamps, int guard, ChainGate G) {
    if (guard && !chain_enter(tmo + 1, tmo + 3)) {   // not co-resident: leave the state to the host's fallback
        chain_leave(tmo + 1, G);
        return;
    }
    constexpr int NT = kChainNT, PER = kChainPer;
    // early (LREC red-black only; the host checked that every halo sub-element is an up one):
    // 1 a sweep's halo words go out right after its up pass, 2 and its flag, 3 as 2 with the up
    // pass split -- item 0 the up sub-elements without halo words (Level::nui per un_ele, first in
    // cpos), run before the wait for the neighbours; item 1 the ones with words, after it
    const bool split = LREC && RB && early == 3;
    __shared__ double X[3][NT * PER];
    __shared__ double HI[kChainHalo];   // this workgroup's un_eles' t_overlap(1 : 3m, 1 : 3) of the sweep
    __shared__ double RS[LREC ? kChainRec * kRecW : 1];
    const int t = threadIdx.x, w = blockIdx.x;
    const int64_t s0 = (int64_t)w * E;
    const int64_t nsm = (1ll << nsub_log2) - 1;
    const int m = H.m, ke = E >> nsub_log2;   // positions along an un_ele face, un_eles of the workgroup
    const int64_t u0 = s0 >> nsub_log2;
    const int nhalo = ke * 9 * m;
    if constexpr (LREC) chain_load_recs(RS, stc, fface, fsx, u0, (int)std::min<int64_t>(ke, (N >> nsub_log2) - u0), t, NT);
    // with LREC the passes run over item lists (red-black: each colour over its positions, all lanes
    // busy; Jacobi: the positions in order), as k_face_wave's
    constexpr int KU = PER, KD = RB ? 1 : 0;
    Items<KU> IA;
    Items<KD == 0 ? 1 : KD> IB;
    if constexpr (LREC) {
        const int kv = (int)std::min<int64_t>(ke, (N >> nsub_log2) - u0), nsub = 1 << nsub_log2;
        const int ndn = nsub - nup;
#pragma unroll
        for (int k = 0; k < KU; ++k) {
            const int i = t + NT * k;
            int j = -1;
            if (RB && split) {
                const int nk = k == 0 ? nui : nup - nui, o = k == 0 ? 0 : nui;
                if (k < 2 && t < kv * nk) {
                    const int uk = t / nk;
                    j = (uk << nsub_log2) + cpos[o + t - uk * nk];
                }
            } else if (RB) {
                if (i < kv * nup) {
                    const int uk = i / nup;
                    j = (uk << nsub_log2) + cpos[i - uk * nup];
                }
            } else if (i < kv * nsub) {
                j = i;
            }
            IA.j[k] = j;
        }
        IB.j[0] = -1;
        if (RB && ndn > 0 && t < kv * ndn) {
            const int uk = t / ndn;
            IB.j[0] = (uk << nsub_log2) + cpos[nup + t - uk * ndn];
        }
        auto fill = [&](auto &I, int K) {
            for (int k = 0; k < K; ++k) {
                const int j = I.j[k] < 0 ? 0 : I.j[k];
                I.nb[k] = fnb[j & nsm];
#pragma unroll
                for (int c = 0; c < 3; ++c) I.b[k][c] = RHS[c * pitch + s0 + j];
            }
        };
        fill(IA, KU);
        if (KD) fill(IB, 1);
    }
    double b[PER][3];
    int4 nbr[PER];
#pragma unroll
    for (int k = 0; k < PER; ++k) {
        const int j = t + NT * k;
        const bool v = j < E && s0 + j < N;
        const int64_t s = v ? s0 + j : s0;
        nbr[k] = fnb[s & nsm];
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            b[k][c] = RHS[c * pitch + s];
            X[c][j] = SRC[c * pitch + s];
        }
    }
    // the halo positions of the thread's pair (2t, 2t + 1), packed 10 bits per face
    int hp[2] = {0, 0};
    if (2 * t < E && s0 + 2 * t < N)
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const int4 e = H.hsub[(s0 + 2 * t + q) & nsm];
            hp[q] = e.x | (e.y << 10) | (e.z << 20);
        }
    __syncthreads();
    auto pass = [&](auto mc) {
        constexpr int MODE = decltype(mc)::value;
        double r[PER][3];
        bool on[PER];
#pragma unroll
        for (int k = 0; k < PER; ++k) {
            const int j = t + NT * k;
            const int64_t s = s0 + j;
            on[k] = false;
            if (j >= E || s >= N) continue;
            int64_t u = s >> nsub_log2;
            if (UNI) u = __builtin_amdgcn_readfirstlane((int)u);
            const int4 nb = nbr[k];
            if ((MODE == 0 && !nb.w) || (MODE == 1 && nb.w)) continue;
            on[k] = true;
            const int jb = (int)((u << nsub_log2) - s0);
            double x[3];
#pragma unroll
            for (int c = 0; c < 3; ++c) x[c] = X[c][j];
            auto xin = [&](int c, int q) { return X[c][jb + q]; };
            auto hv = [&](int64_t uu, int mf, int sp, int kk) {
                return HI[(((int)(uu - u0) * 3 + mf - 1) * m + sp - 1) * 3 + kk];
            };
            face_point<MODE>(xin, x, b[k], nb, u, stc, fface, fsx, hv, level1, rdt, omega, r[k]);
            if (MODE != 2)
#pragma unroll
                for (int c = 0; c < 3; ++c) X[c][j] = r[k][c];
        }
        if (MODE == 2) {
            __syncthreads();
#pragma unroll
            for (int k = 0; k < PER; ++k)
                if (on[k])
#pragma unroll
                    for (int c = 0; c < 3; ++c) X[c][t + NT * k] = r[k][c];
        }
        __syncthreads();
    };
    // the face records of the thread's halo pair's un_ele, fetched once for the call
    int4 hrec[3] = {};
    if ((hp[0] | hp[1]) != 0) {
        const int64_t u = (s0 + 2 * t) >> nsub_log2;
#pragma unroll
        for (int f = 0; f < 3; ++f) hrec[f] = H.hface[3 * u + f];
    }
    // the next sweep's halo words (:550, :555 of sweep sw + 1), written through (sc1)
    auto words = [&](double *tout, int sw) {
        HaloArgs Hn = H;
        Hn.tov = tout;
        const int j = 2 * t;
        // opaque per sweep: the halo destinations are recomputed here instead of hoisted out of the
        // sweep loop (held in registers they spilled)
        int hq[2] = {hp[0], hp[1]};
        int4 hr[3] = {hrec[0], hrec[1], hrec[2]};
        asm volatile("" : "+v"(hq[0]), "+v"(hq[1]));
#pragma unroll
        for (int f = 0; f < 3; ++f) asm volatile("" : "+v"(hr[f].x), "+v"(hr[f].y), "+v"(hr[f].z));
        if ((hq[0] | hq[1]) != 0) {
            // per lane: a wave's pairs span 128 sub-elements, two un_eles when nsub = 64
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                const double tv[3] = {X[0][j + q], X[1][j + q], X[2][j + q]};
                halo_words<true>(Hn, hr, hq[q], tv, sw == 0);
            }
        }
    };
    // tnew := tnew_nonlin (:550) of the call's last sweep, from the tile before that sweep
    auto tstore = [&]() {
#pragma unroll
        for (int k = 0; k < PER; ++k) {
            const int j = t + NT * k;
            if (j < E && s0 + j < N)
#pragma unroll
                for (int c = 0; c < 3; ++c) T[c * pitch + s0 + j] = X[c][j];
        }
    };
    // split: the last sweep's phase A rewrites the tile before the wait, so the store is made
    // from the same values at the end of the sweep before it (or here, for a one-sweep call)
    if (split && store == 1 && run == 1) {
        tstore();
        __syncthreads();
    }
    // the item passes' tile, halo snapshot and un_ele records (LREC)
    auto ixin = [&](int c, int q) { return X[c][q]; };
    auto ihv = [&](int64_t uu, int mf, int sp, int kk) {
        return HI[(((int)(uu - u0) * 3 + mf - 1) * m + sp - 1) * 3 + kk];
    };
    auto irec = [&](int j, int4 nb, auto &&f) { chain_rec(RS, j, nb, nsub_log2, u0, f); };
    // the snapshot's 16-byte loads: a face's 3m words and the slot pitch even (16-byte aligned pairs)
    // (and the snapshot buffer within a buffer resource's 32-bit range; snap_ok = 0 forces the 8-byte
    // form, the path of a larger buffer -- PAMG_CHAIN_SNAP16=0, tests/test_face_operator.py)
    const int64_t tin_bytes64 = (N >> nsub_log2) * slots * 3 * 8;
    const bool snap16 = snap_ok && ((3 * m) & 1) == 0 && (slots & 1) == 0 && tin_bytes64 < (1ll << 31);
    const int tin_bytes = (int)std::min<int64_t>(tin_bytes64, (1ll << 31) - 1);
    const int na = nb_off[w], nn = nb_off[w + 1] - na;
    for (int sw = 0; sw < run; ++sw) {
        const double *tin = ((total - 1 - sw) & 1) ? buf1 : buf0;
        double *tout = sw + 1 < total ? (((total - 2 - sw) & 1) ? buf1 : buf0) : nullptr;
        // diagnostics (PAMG_CHAIN_STAMPS): wall clock at the sweep's start, after the wait and the
        // snapshot's load, after the passes, after the publish -- workgroup 0..7's thread 0
        auto stamp = [&](int i) {
            if (stamps && t == 0 && w < 8) stamps[((int64_t)w * run + sw) * 4 + i] = wall_clock64();
        };
        stamp(0);
        if constexpr (LREC && RB) {
            if (split) {   // the up sub-elements without halo words: no snapshot needed, before the wait
                // (no face of these reads the halo: the snapshot accessor is a constant the compiler drops)
                auto nohv = [](int64_t, int, int, int) { return 0.0; };
                items_pass<0>(IA, ixin, nohv, irec, level1, rdt, [&](int k, const double r[3]) {
#pragma unroll
                    for (int c = 0; c < 3; ++c) X[c][IA.j[k]] = r[c];
                }, 0, 1);
            }
        }
        if (sw > 0 && t < 64) {   // wait for the neighbours' words of this sweep: one wave polls
            for (int base = 0; base < nn; base += 64) {
                const int i = base + t;
                const unsigned *f = i < nn ? flags + nb_list[na + i] : nullptr;
                bool ok = f == nullptr;
                for (unsigned spins = 0;; ++spins) {
                    if (!ok) ok = __hip_atomic_load((g_u32 *)const_cast<unsigned *>(f), __ATOMIC_RELAXED,
                                                    __HIP_MEMORY_SCOPE_AGENT) >= f0 + (unsigned)sw;
                    if (__all(ok)) break;
                    if (spins > (1u << 22)) {
                        if (t == 0) __hip_atomic_store((g_u32 *)tmo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        break;
                    }
                    __builtin_amdgcn_s_sleep(2);
                }
            }
        }
        __syncthreads();
        // the snapshot of this workgroup's un_eles into LDS (every load of the handed-over words
        // through to the coherent level, sc1): 16 bytes a lane where a face's 3m words pair up
        if (snap16) {
            const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<double *>(tin), (short)0, tin_bytes, 0x00020000);
            for (int i2 = t; 2 * i2 < nhalo; i2 += NT) {
                const int idx = 2 * i2;
                const int uk = idx / (9 * m), rem = idx - uk * 9 * m, mf = rem / (3 * m), off = rem - mf * 3 * m;
                const int o = (int)(((u0 + uk) * slots * 3 + (int64_t)mf * slots + off) * 8);
                const v4u v = __builtin_amdgcn_raw_buffer_load_b128(rs, o, 0, kAuxSc1);
                HI[idx] = __longlong_as_double(((long long)v.y << 32) | v.x);
                HI[idx + 1] = __longlong_as_double(((long long)v.w << 32) | v.z);
            }
        } else {
            for (int idx = t; idx < nhalo; idx += NT) {
                const int uk = idx / (9 * m), rem = idx - uk * 9 * m, mf = rem / (3 * m), off = rem - mf * 3 * m;
                HI[idx] = ld_coh(tin + (u0 + uk) * slots * 3 + (int64_t)mf * slots + off);
            }
        }
        // the call's last sweep: tnew := tnew_nonlin (:550), before the barrier that lets the passes
        // rewrite X (with item lists a position's item may belong to another thread)
        if (store == 1 && sw + 1 == run && !split) tstore();
        __syncthreads();
        stamp(1);
        if constexpr (LREC) {
#pragma unroll
            for (int k = 0; k < KU; ++k) asm volatile("" : "+v"(IA.j[k]), "+v"(IA.nb[k].x), "+v"(IA.nb[k].y), "+v"(IA.nb[k].z), "+v"(IA.nb[k].w));
            asm volatile("" : "+v"(IB.j[0]), "+v"(IB.nb[0].x), "+v"(IB.nb[0].y), "+v"(IB.nb[0].z), "+v"(IB.nb[0].w));
            if constexpr (RB) {   // up sub-elements, then down ones, in place
                auto up = [&](int k, const double r[3]) {
#pragma unroll
                    for (int c = 0; c < 3; ++c) X[c][IA.j[k]] = r[c];
                };
                items_pass<0>(IA, ixin, ihv, irec, level1, rdt, up, split ? 1 : 0);   // split: the items with words
                __syncthreads();
                // early: every halo sub-element is an up one (the host checked), final after the
                // up pass -- its words go out now, their write-through latency under the down pass
                if (early && tout) {
                    words(tout, sw);
                    if (early >= 2) {   // and the flag too: the down pass runs while the neighbours read
                        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                        __syncthreads();
                        if (t == 0)
                            __hip_atomic_store((g_u32 *)flags + w, f0 + (unsigned)(sw + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    }
                }
                items_pass<1>(IB, ixin, ihv, irec, level1, rdt, [&](int k, const double r[3]) {
#pragma unroll
                    for (int c = 0; c < 3; ++c) X[c][IB.j[k]] = r[c];
                });
            } else {   // Jacobi: every read of the old iterate before any write
                double rj[KU][3];
                items_pass<2>(IA, ixin, ihv, irec, level1, rdt, [&](int k, const double r[3]) {
#pragma unroll
                    for (int c = 0; c < 3; ++c) rj[k][c] = r[c];
                });
                __syncthreads();
#pragma unroll
                for (int k = 0; k < KU; ++k)
                    if (IA.j[k] >= 0)
#pragma unroll
                        for (int c = 0; c < 3; ++c) X[c][IA.j[k]] = rj[k][c];
            }
            __syncthreads();
            if (split && store == 1 && sw + 2 == run) {   // the last sweep's tnew (see tstore)
                tstore();
                __syncthreads();
            }
        } else if constexpr (RB) {
            pass(std::integral_constant<int, 0>{});
            pass(std::integral_constant<int, 1>{});
        } else {
            pass(std::integral_constant<int, 2>{});
        }
        stamp(2);
        if (tout && !(LREC && RB && early >= 2)) {   // publish: every storing wave drains, then the workgroup's flag
            if (!(LREC && RB && early)) words(tout, sw);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (t == 0) __hip_atomic_store((g_u32 *)flags + w, f0 + (unsigned)(sw + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        stamp(3);
    }
#pragma unroll
    for (int k = 0; k < PER; ++k) {   // tnew_nonlin (store 2: tnew, the dead last sweep's :550; 3: both)
        const int j = t + NT * k;
        if (j < E && s0 + j < N)
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                if (store != 2) TNN[c * pitch + s0 + j] = X[c][j];
                if (store >= 2) T[c * pitch + s0 + j] = X[c][j];
            }
    }
    if (guard) chain_leave(tmo + 1, G);
}

// ---- the chain with un_eles owned by waves (PAMG_CHAIN_PW, default where it applies): the red-black
// sweep of an un_ele reads, besides the halo snapshot, only its own sub-elements -- an up one its down
// neighbours, a down one its up neighbours -- so each wave of the workgroup takes q = k / 16 whole un_eles
// and runs their passes without the workgroup: item 0 (the ups without halo words), the wait for the
// words of the previous sweep, the snapshot of its own un_eles, item 1 (the ups with words, whose words
// for the next sweep it writes at once), the drain, its own flag, the down pass. A wave's LDS writes are
// read only by that wave (its un_eles' slots of X and HI), in order; the records are loaded behind the
// one barrier of the launch. Flags are per wave (flags[16 w + v]); a wave waits for the 16 waves of its
// own workgroup and of every neighbouring workgroup (a superset of the waves owning its un_eles'
// neighbours). The buffer argument is the workgroup chain's: a wave writes snapshot buffer (s + 1) & 1
// only after every wave that reads its words there has published sweep s - 1, i.e. loaded the snapshot
// of sweep s - 1 from it. Same items, same face_apply on the same operands in the same colour order:
// bitwise k_face_chain (tests/test_face_operator.py). Needs every halo sub-element to be an up one
// (words_up) and q un_eles' colour lists in 64 lanes (level 3 at n_split = 5: 2 x 15, 2 x 21, 2 x 28).
constexpr int kPW = kChainNT / 64;   // waves of a chain workgroup
constexpr int kPWStamps = 7;         // per-wave phase stamps a sweep (PAMG_CHAIN_STAMPS)
__global__ __launch_bounds__(kChainNT, 1) void k_face_chain_pw(double *T, double *TNN, const double *SRC,
                                                               const double *__restrict__ RHS,
                                                               const double *__restrict__ stc, const int4 *__restrict__ fnb,
                                                               const double *__restrict__ fface, const int *__restrict__ fsx,
                                                               double *buf0, double *buf1, HaloArgs H, unsigned *flags,
                                                               const int *__restrict__ nb_off, const int *__restrict__ nb_list,
                                                               unsigned *tmo, int run, int total, int store, int E,
                                                               int64_t pitch, int64_t N, int nsub_log2, int slots, int level1,
                                                               double rdt, double omega, const int *__restrict__ cpos,
                                                               int nup, int nui, int early, unsigned f0, int snap_ok,
                                                               long long *stamps, int guard, ChainGate G) {
    (void)omega;
    if (guard && !chain_enter(tmo + 1, tmo + 3)) {   // not co-resident: leave the state to the host's fallback
        chain_leave(tmo + 1, G);
        return;
    }
    constexpr int NT = kChainNT;
    // one LDS image: the iterate planes (X), the halo snapshot (HI), the records (RS) and a zero word, so that an
    // item's operands are one index each (pw_face below)
    constexpr int XP = NT * kChainPer, OHI = 3 * XP, ORS = OHI + kChainHalo, OZ = ORS + kChainRec * kRecW;
    static_assert(OZ < (1 << 15), "15-bit operand indices");
    __shared__ double LM[OZ + 1];
    __shared__ unsigned wgc, wgready, wgpoll;   // the workgroup's published waves, ready sweep, polling claim
    const int t = threadIdx.x, w = blockIdx.x;
    const int v = __builtin_amdgcn_readfirstlane(t >> 6), ln = t & 63;
    // flags (early bits 32 / 64; PAMG_CHAIN_WGFLAG, default 2): 0 one flag per wave (flags[16 w + v]), a wave
    // polls the 16 (nn + 1) flags of its own and the neighbouring workgroups; 1 one flag per workgroup
    // (flags[16 w]), stored by the last of its 16 waves to publish -- each wave drains its words, then adds to
    // the LDS counter wgc, the last arriver stores the flag (Guideline 16 R1's counter form) -- and a wave polls
    // nn + 1 flags; 2 as 1, with one wave of the workgroup polling (the first to arrive, claimed in wgpoll) and
    // the others waiting on its LDS word wgready
    const bool wgflag = (early & 32) != 0, leader_poll = (early & 64) != 0;
    if (t == 0) {
        wgc = 0;
        wgready = 0;
        wgpoll = 0;
        LM[OZ] = 0.0;
    }
    const int64_t s0 = (int64_t)w * E;
    const int64_t nsm = (1ll << nsub_log2) - 1;
    const int m = H.m, ke = E >> nsub_log2;
    const int64_t u0 = s0 >> nsub_log2;
    const int kv = (int)std::min<int64_t>(ke, (N >> nsub_log2) - u0);
    const int q = (ke + kPW - 1) / kPW;                  // un_eles per wave
    const int ua = std::min(kv, v * q), ub = std::min(kv, ua + q);   // this wave's un_eles [ua, ub)
    const int nsub = 1 << nsub_log2, ndn = nsub - nup, n1 = nup - nui;
    chain_load_recs(LM + ORS, stc, fface, fsx, u0, kv, t, NT);   // the un_eles' records
    // the lane's items: 0 an up sub-element without halo words, 1 one with words, D a down one
    Items<1> I0, I1, ID;
    auto mk = [&](Items<1> &I, int n, int o) {
        const int uk = n > 0 ? ua + ln / n : ub;
        I.j[0] = (n > 0 && ln < q * n && uk < ub) ? (uk << nsub_log2) + cpos[o + ln % n] : -1;
        const int j = I.j[0] < 0 ? 0 : I.j[0];
        I.nb[0] = fnb[j & nsm];
#pragma unroll
        for (int c = 0; c < 3; ++c) I.b[0][c] = RHS[c * pitch + s0 + j];
    };
    mk(I0, nui, 0);
    mk(I1, n1, nui);
    mk(ID, ndn, nup);
    // item 1's halo positions (packed 10 bits per face) and its un_ele's face records
    int hq = 0;
    int4 hr[3] = {};
    if (I1.j[0] >= 0) {
        const int4 e = H.hsub[I1.j[0] & nsm];
        hq = e.x | (e.y << 10) | (e.z << 20);
        const int64_t u = u0 + (I1.j[0] >> nsub_log2);
#pragma unroll
        for (int f = 0; f < 3; ++f) hr[f] = H.hface[3 * u + f];
    }
    const int pa = ua << nsub_log2, pb = ub << nsub_log2;   // the wave's tile positions
    for (int j = pa + ln; j < pb; j += 64)
#pragma unroll
        for (int c = 0; c < 3; ++c) LM[c * XP + j] = SRC[c * pitch + s0 + j];
    __syncthreads();   // the records
    // An item's operands, fixed for the call: per sub-element face fi the LM indices of the two values face_apply
    // reads there (ya, yb: the inner neighbour's components fnode(fi, 1), fnode(fi, 0), or the halo snapshot's
    // selected words, or the zero word for a coarse level's homogeneous boundary) and whether the face is inner,
    // packed 15 + 15 + 1 bits -- so a pass issues every LDS read of its item at once instead of a branch per face
    // with its own reads and waits (the item-1 pass is on the chain's critical path). face_apply's arithmetic on
    // the same values in the same order: bitwise (tests/test_face_operator.py).
    auto pack = [&](const Items<1> &I, unsigned P[3]) {
        const int j = I.j[0] < 0 ? 0 : I.j[0], uk = j >> nsub_log2, jb = uk << nsub_log2;
        const int nbf[3] = {I.nb[0].x, I.nb[0].y, I.nb[0].z};
#pragma unroll
        for (int fi = 0; fi < 3; ++fi) {
            const int a = fnode(fi, 0), bb = fnode(fi, 1);
            int ia, ib;
            if (nbf[fi] >= 0) {
                ia = bb * XP + jb + nbf[fi];
                ib = a * XP + jb + nbf[fi];
            } else {
                const int sx = (int)LM[ORS + uk * kRecW + 43 + fi];
                const int h = OHI + ((uk * 3 + fmface(fi) - 1) * m - nbf[fi] - 1) * 3;
                if (!level1 && (sx & 16)) ia = ib = OZ;
                else {
                    ia = h + (sx & 3) - 1;
                    ib = h + ((sx >> 2) & 3) - 1;
                }
            }
            P[fi] = (unsigned)ia | ((unsigned)ib << 15) | ((nbf[fi] >= 0 ? 1u : 0u) << 30);
        }
    };
    unsigned P0[3], P1[3], PD[3];
    pack(I0, P0);
    pack(I1, P1);
    pack(ID, PD);
    // one item: face_apply<0 / 1> (the smoother update) of tile position j from its record, its packed operands
    auto pw_face = [&](int j, const unsigned P[3], const double b[3], double r[3]) {
        const double *rs = LM + ORS + (j >> nsub_log2) * kRecW;
        double x[3], y[3][2], wf[3];
#pragma unroll
        for (int c = 0; c < 3; ++c) x[c] = LM[c * XP + j];
#pragma unroll
        for (int fi = 0; fi < 3; ++fi) {
            y[fi][0] = LM[P[fi] & 32767];
            y[fi][1] = LM[(P[fi] >> 15) & 32767];
        }
        Stc S;
        S.c = rs[0];
#pragma unroll
        for (int k = 0; k < 9; ++k) S.K[k] = rs[1 + k];
        const int pat = (int)((P[0] >> 30) | ((P[1] >> 30) << 1) | ((P[2] >> 30) << 2));
#pragma unroll
        for (int fi = 0; fi < 3; ++fi) wf[fi] = (P[fi] >> 30) ? rs[13 + fi] : rs[13 + 3 + fmface(fi) - 1];
        const double *wd = rs + 19 + 3 * pat;
        double A[3];
        apply_A(S, rdt, x, A);
        double ds[3] = {0.0, 0.0, 0.0};
#pragma unroll
        for (int fi = 0; fi < 3; ++fi) {
            const int a = fnode(fi, 0), bb = fnode(fi, 1);
            const double ya = y[fi][0], yb = y[fi][1];
            ds[a] = ds[a] + wf[fi] * (((2.0 * x[a] + x[bb]) - 2.0 * ya) - yb);
            ds[bb] = ds[bb] + wf[fi] * (((x[a] + 2.0 * x[bb]) - ya) - 2.0 * yb);
        }
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            const double ai = A[i] + ds[i];
            r[i] = x[i] + wd[i] * (b[i] - ai);
        }
    };
    auto tstore = [&]() {
        for (int j = pa + ln; j < pb; j += 64)
#pragma unroll
            for (int c = 0; c < 3; ++c) T[c * pitch + s0 + j] = LM[c * XP + j];
    };
    if (store == 1 && run == 1) tstore();
    const int64_t tin_bytes64 = (N >> nsub_log2) * slots * 3 * 8;
    const bool snap16 = snap_ok && ((3 * m) & 1) == 0 && (slots & 1) == 0 && tin_bytes64 < (1ll << 31);
    const int tin_bytes = (int)std::min<int64_t>(tin_bytes64, (1ll << 31) - 1);
    const int na = nb_off[w], nn = nb_off[w + 1] - na;
    const int ha = ua * 9 * m, hb = ub * 9 * m;   // the wave's slots of the snapshot image
    // the snapshot loads' byte offsets (the same every sweep: only the buffer alternates) when a lane
    // has at most two (two un_eles of m = 8: 144 words, 72 pairs), so the sweep does no index division
    const bool snap_pre = snap16 && hb - ha <= 256;
    int so[2] = {-1, -1};
    if (snap_pre)
#pragma unroll
        for (int it = 0; it < 2; ++it) {
            const int idx = ha + 2 * ln + 128 * it;
            if (idx >= hb) continue;
            const int uk = idx / (9 * m), rem = idx - uk * 9 * m, mf = rem / (3 * m), off = rem - mf * 3 * m;
            so[it] = (int)(((u0 + uk) * slots * 3 + (int64_t)mf * slots + off) * 8);
        }
    // Coalesced words (cw): a sweep's halo words leave as 16-byte sc1 buffer stores of whole t_overlap rows (Guideline
    // 16 R1's payload form) instead of three 8-byte stores per face from each item-1 lane: the wave's rows (its
    // un_eles' faces to neighbours on this rank, 3m words each) are cut into 16-byte chunks, a lane takes one or two
    // and reads their two words from the tile in LDS, where the item-1 pass has just put them (this wave's own lanes).
    // Word w of a row is component w % 3 of the sub-element at face position i (k = w / 3 + 1, i = k or m + 1 - k
    // reversed: halo_words' placement inverted). Per lane, fixed for the call: the chunk's byte offset in a snapshot
    // buffer and its two LDS indices. The boundary faces' constant words go out once, before the sweeps, into the
    // buffer the first sweep writes (as halo_words with bc there).
    const int rowc = 3 * m / 2, nch = (ub - ua) * 3 * rowc;
    const bool cw = snap16 && nch <= 128 && 3 * m <= 9 * m * (ub - ua);
    int co[2] = {-1, -1};
    unsigned ci[2] = {0u, 0u};
    if (cw) {
        // face position -> tile-local sub-element (the same in every un_ele of the level), in this wave's slots of
        // the snapshot image as scratch until the first snapshot load
        for (int j = ln; j < nsub; j += 64) {
            const int4 e = H.hsub[j];
            if (e.x) LM[OHI + ha + e.x - 1] = (double)j;
            if (e.y) LM[OHI + ha + m + e.y - 1] = (double)j;
            if (e.z) LM[OHI + ha + 2 * m + e.z - 1] = (double)j;
        }
#pragma unroll
        for (int it = 0; it < 2; ++it) {
            const int ch = ln + 64 * it;
            if (ch >= nch) continue;
            const int uk = ua + ch / (3 * rowc), rem = ch % (3 * rowc), f = rem / rowc, cwi = rem % rowc;
            const int4 rec = H.hface[3 * (u0 + uk) + f];
            if ((rec.x & 3) != 1) continue;
            const bool rev = (rec.x >> 2) != 0;
            unsigned idx[2];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int w = 2 * cwi + h, k = w / 3 + 1, c = w % 3, i = rev ? m - k + 1 : k;
                const int j = (int)LM[OHI + ha + f * m + i - 1];
                idx[h] = (unsigned)(c * XP + (uk << nsub_log2) + j);
            }
            ci[it] = idx[0] | (idx[1] << 16);
            co[it] = (rec.y + 2 * cwi) * 8;
        }
        // the boundary faces' words, constant in the call, into the buffer the first sweep publishes into
        if (run >= 1 && 1 < total && I1.j[0] >= 0) {
            double *tout0 = ((total - 2) & 1) ? buf1 : buf0;
            const int pos[3] = {hq & 1023, (hq >> 10) & 1023, hq >> 20};
#pragma unroll
            for (int f = 0; f < 3; ++f) {
                const int i = pos[f];
                if (!i || (hr[f].x & 3) != 0) continue;
                const int a = (i - 1) * 3 + (f == 2 ? 1 : 0), b = (i - 1) * 3 + (f == 1 ? 1 : 2);
                const double2 v = H.bcv[hr[f].z + i - 1];
                st_coh(tout0 + hr[f].y + a, v.x);
                st_coh(tout0 + hr[f].y + b, v.y);
            }
        }
    }
    // poll flags f[0 .. n) (lane i one) until each is >= want; bounded (the give-up word tmo)
    auto poll = [&](int n, auto &&flag_of, unsigned want) {
        for (int base = 0; base < n; base += 64) {
            const int i = base + ln;
            const unsigned *f = i < n ? flag_of(i) : nullptr;
            bool ok = f == nullptr;
            for (unsigned spins = 0;; ++spins) {
                if (!ok) ok = __hip_atomic_load((g_u32 *)const_cast<unsigned *>(f), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= want;
                if (__all(ok)) break;
                if (spins > (1u << 22)) {
                    if (ln == 0) __hip_atomic_store((g_u32 *)tmo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    break;
                }
                __builtin_amdgcn_s_sleep(2);
            }
        }
    };
    auto wg_flag = [&](int i) { return flags + (size_t)(i == 0 ? w : nb_list[na + i - 1]) * kPW; };
    for (int sw = 0; sw < run; ++sw) {
        const double *tin = ((total - 1 - sw) & 1) ? buf1 : buf0;
        double *tout = sw + 1 < total ? (((total - 2 - sw) & 1) ? buf1 : buf0) : nullptr;
        // PAMG_CHAIN_STAMPS: per-wave phase stamps of workgroups 0..7 (kPWStamps a sweep)
        auto stamp = [&](int i) {
            if (stamps && ln == 0 && w < 8) stamps[(((int64_t)w * kPW + v) * run + sw) * kPWStamps + i] = wall_clock64();
        };
        stamp(0);
        // opaque per sweep (as k_face_chain's): the items stay in their registers instead of being
        // rematerialized or hoisted around the passes
        asm volatile("" : "+v"(I0.j[0]), "+v"(P0[0]), "+v"(P0[1]), "+v"(P0[2]));
        asm volatile("" : "+v"(I1.j[0]), "+v"(P1[0]), "+v"(P1[1]), "+v"(P1[2]));
        asm volatile("" : "+v"(ID.j[0]), "+v"(PD[0]), "+v"(PD[1]), "+v"(PD[2]));
        asm volatile("" : "+v"(hq));
#pragma unroll
        for (int f = 0; f < 3; ++f) asm volatile("" : "+v"(hr[f].x), "+v"(hr[f].y), "+v"(hr[f].z));
        if (I0.j[0] >= 0) {
            double r[3];
            pw_face(I0.j[0], P0, I0.b[0], r);
#pragma unroll
            for (int c = 0; c < 3; ++c) LM[c * XP + I0.j[0]] = r[c];
        }
        stamp(1);
        if (sw > 0 && wgflag && leader_poll) {   // one wave polls the workgroup flags, the others its LDS word
            if (__hip_atomic_load(&wgready, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < (unsigned)sw) {
                unsigned old = 0;
                if (ln == 0) old = __hip_atomic_fetch_max(&wgpoll, (unsigned)sw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                old = __builtin_amdgcn_readfirstlane(old);
                if (old < (unsigned)sw) {
                    poll(nn + 1, wg_flag, f0 + (unsigned)sw);
                    if (ln == 0) __hip_atomic_fetch_max(&wgready, (unsigned)sw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                } else {
                    for (unsigned spins = 0;; ++spins) {
                        if (__hip_atomic_load(&wgready, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) >= (unsigned)sw) break;
                        if (spins > (1u << 27)) {   // the poller gives up after 2^22 polls (>= 4 s) and still releases this word
                            if (ln == 0) __hip_atomic_store((g_u32 *)tmo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                            break;
                        }
                        __builtin_amdgcn_s_sleep(1);
                    }
                }
            }
        } else if (sw > 0 && wgflag) {   // the workgroup flags of this and of the neighbouring workgroups
            poll(nn + 1, wg_flag, f0 + (unsigned)sw);
        } else if (sw > 0) {   // every wave of this and of the neighbouring workgroups has published sweep sw - 1
            poll((nn + 1) * kPW, [&](int i) { const int g = i / kPW; return wg_flag(g) + (i - g * kPW); }, f0 + (unsigned)sw);
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   // no instruction: the snapshot loads stay below the wait
        stamp(2);
        // the snapshot of the wave's un_eles (sc1: through to the coherent level)
        if (snap_pre) {   // at most two 16-byte loads a lane, their offsets computed once for the call
            asm volatile("" : "+v"(so[0]), "+v"(so[1]));
            const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<double *>(tin), (short)0, tin_bytes, 0x00020000);
#pragma unroll
            for (int it = 0; it < 2; ++it) {
                if (so[it] < 0) continue;
                const int idx = ha + 2 * ln + 128 * it;
                const v4u val = __builtin_amdgcn_raw_buffer_load_b128(rs, so[it], 0, kAuxSc1);
                LM[OHI + idx] = __longlong_as_double(((long long)val.y << 32) | val.x);
                LM[OHI + idx + 1] = __longlong_as_double(((long long)val.w << 32) | val.z);
            }
        } else if (snap16) {
            const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<double *>(tin), (short)0, tin_bytes, 0x00020000);
            for (int idx = ha + 2 * ln; idx < hb; idx += 128) {
                const int uk = idx / (9 * m), rem = idx - uk * 9 * m, mf = rem / (3 * m), off = rem - mf * 3 * m;
                const int o = (int)(((u0 + uk) * slots * 3 + (int64_t)mf * slots + off) * 8);
                const v4u val = __builtin_amdgcn_raw_buffer_load_b128(rs, o, 0, kAuxSc1);
                LM[OHI + idx] = __longlong_as_double(((long long)val.y << 32) | val.x);
                LM[OHI + idx + 1] = __longlong_as_double(((long long)val.w << 32) | val.z);
            }
        } else {
            for (int idx = ha + ln; idx < hb; idx += 64) {
                const int uk = idx / (9 * m), rem = idx - uk * 9 * m, mf = rem / (3 * m), off = rem - mf * 3 * m;
                LM[OHI + idx] = ld_coh(tin + (u0 + uk) * slots * 3 + (int64_t)mf * slots + off);
            }
        }
        if (stamps) {
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
            stamp(3);
        }
        // the ups with words, their next-sweep words written through at once
        if (I1.j[0] >= 0) {
            double r[3];
            pw_face(I1.j[0], P1, I1.b[0], r);
#pragma unroll
            for (int c = 0; c < 3; ++c) LM[c * XP + I1.j[0]] = r[c];
            if (tout && !cw) {
                HaloArgs Hn = H;
                Hn.tov = tout;
                halo_words<true>(Hn, hr, hq, r, sw == 0);
            }
        }
        if (tout && cw) {   // this wave's rows, 16 bytes a lane (the item-1 values just written to LM)
            asm volatile("" : "+v"(co[0]), "+v"(co[1]), "+v"(ci[0]), "+v"(ci[1]));
            const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(tout, (short)0, tin_bytes, 0x00020000);
#pragma unroll
            for (int it = 0; it < 2; ++it) {
                if (co[it] < 0) continue;
                const double v0 = LM[ci[it] & 65535], v1 = LM[ci[it] >> 16];
                const unsigned long long b0 = (unsigned long long)__double_as_longlong(v0),
                                         b1 = (unsigned long long)__double_as_longlong(v1);
                const v4u val = {(unsigned)b0, (unsigned)(b0 >> 32), (unsigned)b1, (unsigned)(b1 >> 32)};
                __builtin_amdgcn_raw_buffer_store_b128(val, rs, co[it], 0, kAuxSc1);
            }
        }
        if (stamps) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            stamp(4);
        }
        if (tout) {   // drained, then this wave's flag (wgflag: the workgroup's, by its last wave)
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if (wgflag) {
                if (ln == 0 && __hip_atomic_fetch_add(&wgc, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) + 1 ==
                                   (unsigned)kPW * (unsigned)(sw + 1))
                    __hip_atomic_store((g_u32 *)flags + (size_t)w * kPW, f0 + (unsigned)(sw + 1), __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
            } else if (ln == 0) {
                __hip_atomic_store((g_u32 *)flags + (size_t)w * kPW + v, f0 + (unsigned)(sw + 1), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        stamp(5);
        if (ID.j[0] >= 0) {
            double r[3];
            pw_face(ID.j[0], PD, ID.b[0], r);
#pragma unroll
            for (int c = 0; c < 3; ++c) LM[c * XP + ID.j[0]] = r[c];
        }
        if (stamps) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            stamp(6);
        }
        if (store == 1 && sw + 2 == run) tstore();   // the last sweep's tnew := tnew_nonlin (its start)
    }
    for (int j = pa + ln; j < pb; j += 64)   // tnew_nonlin (store 2: tnew, the dead last sweep's :550; 3: both)
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            if (store != 2) TNN[c * pitch + s0 + j] = LM[c * XP + j];
            if (store >= 2) T[c * pitch + s0 + j] = LM[c * XP + j];
        }
    if (guard) chain_leave(tmo + 1, G);
}

inline unsigned grid_for(int64_t n) { return (unsigned)((n + kBlock - 1) / kBlock); }
inline int log2i(int v) { int r = 0; while ((1 << r) < v) ++r; return r; }

}  // namespace

hipError_t launch_face_halo(hipStream_t s, const Level &L, double *tov, double *tovo, bool copy) {
    const int64_t npairs = L.N / 2;
    if (npairs == 0) return hipSuccess;
    const HaloPlan &P = L.halo;
    HaloArgs H{P.d_hsub, P.d_hface, P.d_bcv, P.d_told_halo, tov, tovo, P.d_send, 1 << L.isplit};
    hipLaunchKernelGGL(k_face_halo, dim3(grid_for(npairs)), dim3(kBlock), 0, s, L.T, L.TNN, L.pitch, npairs,
                       log2i(L.nsub), H, copy ? 1 : 0);
    return hipGetLastError();
}

hipError_t launch_face_words(hipStream_t s, const Level &L, int U, double *tov, double *tovo) {
    const HaloPlan &P = L.halo;
    const int64_t nwork = (int64_t)U * P.nbpos;
    if (nwork == 0 || L.N == 0) return hipSuccess;
    HaloArgs H{P.d_hsub, P.d_hface, P.d_bcv, P.d_told_halo, tov, tovo, P.d_send, 1 << L.isplit};
    hipLaunchKernelGGL(k_face_words, dim3(grid_for(nwork)), dim3(kBlock), 0, s, L.T, L.pitch, H, P.d_bpos, P.nbpos,
                       nwork, log2i(L.nsub));
    return hipGetLastError();
}

hipError_t launch_face_sweep(hipStream_t s, const Level &L, const double *tov, int mode, bool level1, double rdt,
                             double omega, int slots) {
    if (L.N == 0) return hipSuccess;
    if (!L.fnb || !L.fface || !L.fsx) return hipErrorInvalidValue;
    const dim3 g(grid_for(L.N)), b(kBlock);
    const int lg = log2i(L.nsub), l1 = level1 ? 1 : 0;
    const bool uni = L.nsub >= 64;
#define PAMG_FACE(M, X_, O_)                                                                                        \
    if (uni) hipLaunchKernelGGL((k_face<M, true>), g, b, 0, s, X_, O_, L.RHS, L.stc, L.fnb, L.fface, L.fsx, tov,     \
                                L.pitch, L.N, lg, slots, l1, rdt, omega);                                           \
    else hipLaunchKernelGGL((k_face<M, false>), g, b, 0, s, X_, O_, L.RHS, L.stc, L.fnb, L.fface, L.fsx, tov,       \
                            L.pitch, L.N, lg, slots, l1, rdt, omega)
    switch (mode) {
        case 0: PAMG_FACE(0, L.TNN, L.TNN); break;
        case 1: PAMG_FACE(1, L.TNN, L.TNN); break;
        case 2: PAMG_FACE(2, L.T, L.TNN); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// the levels whose sweep is one tile per un_ele (k_face_tile: 256, 1,024 or 4,096 sub-elements)
bool face_tile_shape(const Level &L) { return (L.nsub == 256 || L.nsub == 1024 || L.nsub == 4096) && L.N % L.nsub == 0; }

// one fused sweep (k_face_sweep): reads the halo snapshot tin, writes the next sweep's halo words
// into tout unless tout is null; single domain, un_eles of at most 4096 sub-elements
bool face_sweep_fusable(const Level &L) { return L.nsub <= 4096; }

hipError_t launch_face_sweep_fused(hipStream_t s, const Level &L, const double *tin, double *tout, double *tovo,
                                   bool rb, bool level1, double rdt, double omega, int slots, int store, bool bc,
                                   bool from_T, double *res) {
    if (L.N == 0) return hipSuccess;
    const double *src = from_T ? L.T : L.TNN;   // the sweep's iterate (from_T: tnew holds tnew_nonlin)
    if (!L.fnb || !L.fface || !L.fsx || !face_sweep_fusable(L)) return hipErrorInvalidValue;
    const HaloPlan &P = L.halo;
    HaloArgs H{P.d_hsub, P.d_hface, P.d_bcv, P.d_told_halo, tout, tovo, P.d_send, 1 << L.isplit};
    const int lg = log2i(L.nsub), l1 = level1 ? 1 : 0, nh = tout ? 1 : 0, st = store;
    const bool uni = L.nsub >= 64;
#define PAMG_FSW(TS, NT, U, R)                                                                                      \
    hipLaunchKernelGGL((k_face_sweep<TS, NT, U, R>), dim3((unsigned)((L.N + TS - 1) / TS)), dim3(NT), 0, s, L.T,   \
                       L.TNN, src, L.RHS, L.stc, L.fnb, L.fface, L.fsx, tin, H, nh, st, L.pitch, L.N, lg, slots, l1, rdt, \
                       omega)
    // un_eles of 256, 1,024 or 4,096 sub-elements: one tile per un_ele (k_face_tile); the smaller
    // ones in tiles of 256 (more workgroups per CU for sweeps that are short and latency-bound)
    if (res && !face_tile_shape(L)) return hipErrorInvalidValue;
    if (face_tile_shape(L)) {
        const dim3 g((unsigned)(L.N / L.nsub));
        const int b = bc ? 1 : 0;
#define PAMG_FTL(TS, NT, R)                                                                                         \
    hipLaunchKernelGGL((k_face_tile<TS, NT, R>), g, dim3(NT), 0, s, L.T, L.TNN, src, L.RHS, L.stc, L.fnb, L.fface, L.fsx, \
                       tin, H, nh, b, st, L.pitch, slots, l1, rdt, res)
        if (L.nsub == 4096) {
            if (rb) PAMG_FTL(4096, 1024, true);
            else PAMG_FTL(4096, 1024, false);
        } else if (L.nsub == 1024) {
            if (rb) PAMG_FTL(1024, 512, true);
            else PAMG_FTL(1024, 512, false);
        } else {
            if (rb) PAMG_FTL(256, 128, true);
            else PAMG_FTL(256, 128, false);
        }
#undef PAMG_FTL
    } else if (L.nsub > 1024) {
        if (rb) PAMG_FSW(4096, 1024, true, true);
        else PAMG_FSW(4096, 1024, true, false);
    } else if (uni) {
        if (rb) PAMG_FSW(256, 128, true, true);
        else PAMG_FSW(256, 128, true, false);
    } else {
        if (rb) PAMG_FSW(256, 128, false, true);
        else PAMG_FSW(256, 128, false, false);
    }
#undef PAMG_FSW
    return hipGetLastError();
}

// Launch of a grid whose workgroups wait on each other (k_face_chain, k_face_wave): it must be resident
// at once. hipLaunchCooperativeKernel checks that, but a process that used it crashed at exit under
// rocprofv3's kernel trace -- SIGSEGV inside libhsa-runtime64, called from libamdhip64's exit-time
// teardown, on a GPU mapping already gone (profiles/r04_a_face_exit.txt; the same probe without the
// chain exits cleanly). So the grid is checked against the same occupancy bound the cooperative launch
// checks (workgroups per CU x CUs) and launched as a plain kernel: on the stream's turn every workgroup
// of such a grid is dispatched at once, and every in-kernel wait is bounded (the give-up word tmo), so a
// grid that did not become resident ends in PAMG_ERR_HIP, never in a hang (round 5: the arrival guard
// makes such a grid leave without touching anything, and the host runs the call's fallback).
static hipError_t launch_coresident(const void *f, int grid, int nt, void **args, hipStream_t s) {
    static std::mutex mu;
    static std::map<std::pair<const void *, int>, int> cap;   // co-resident workgroups per (kernel, block)
    int n = 0;
    {
        std::lock_guard<std::mutex> lk(mu);
        auto it = cap.find({f, nt});
        if (it == cap.end()) {
            int dev = 0, cus = 0, per = 0;
            hipError_t e = hipGetDevice(&dev);
            if (e == hipSuccess) e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
            if (e == hipSuccess) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, f, nt, 0);
            if (e != hipSuccess) return e;
            it = cap.emplace(std::make_pair(f, nt), per * cus).first;
        }
        n = it->second;
    }
    if (grid > n) return hipErrorCooperativeLaunchTooLarge;
    return hipLaunchKernel(f, dim3(grid), dim3(nt), args, 0, s);
}

// k_face_pp: K sweeps of a whole-un_ele-tile level in one launch (face_tile_shape; single domain)
hipError_t launch_face_pp(hipStream_t s, const Level &L, int K, const double *in, double *out_pre, double *out_mid,
                          double *out_end, bool rb, bool level1, double rdt, int res, double *out_end2, const PPCoarse *pcx) {
    if (L.N == 0) return hipSuccess;
    const int m = L.nsub == 256 ? 16 : L.nsub == 1024 ? 32 : 64;
    if (!face_tile_shape(L) || !L.fnb || !L.gtab || !L.gpat || (K != 1 && K != 2) || (K == 1 && (out_mid || res == 2)) ||
        (out_end2 && (out_end2 == in || !out_end)) ||
        (rb && (!L.cpos || !L.cnb || L.nup != m * (m + 1) / 2)))
        return hipErrorInvalidValue;
    // the coarse level (pcx): this one's quarter, the same un_eles, 4 children per coarse sub-element
    const Level *C = pcx ? pcx->coarse : nullptr;
    if (pcx && (!C || C->N * 4 != L.N)) return hipErrorInvalidValue;
    const bool interp = pcx && pcx->interp;
    double *RC = pcx ? pcx->rhsc : nullptr;
    // res 3: the residual restricted into the coarse RHS, one sweep-less pass (K 1, no iterate outputs); a
    // restriction needs a residual; interp: the start iterate in + the prolonged correction of the coarse level's T;
    // in null: a start from zero
    if ((res == 3 && (K != 1 || out_pre || out_end || out_end2 || !RC)) || (RC && !res) ||
        (interp && (res == 3 || !in || !C->T)) || (!in && res))
        return hipErrorInvalidValue;
    const HaloPlan &P = L.halo;
    const dim3 g((unsigned)(L.N / L.nsub));
    const int l1 = level1 ? 1 : 0;
    double *R = res && (!pcx || pcx->res_store) ? L.RES : nullptr;
    if (res && !R && !RC) return hipErrorInvalidValue;
    const double *TC = interp ? C->T : nullptr;
    const int64_t pc = C ? C->pitch : 0;
    // PAMG_PP_STAMPS=<file> (a PAMG_STAMPS=1 build): append each launch's per-workgroup phase stamps
    static const char *stamp_path = PAMG_STAMPS ? getenv("PAMG_PP_STAMPS") : nullptr;
    long long *stamps = nullptr;
    const size_t nst = (size_t)g.x * kPPStamps;
    if (stamp_path) {
        hipError_t e = hipMalloc(&stamps, nst * sizeof(long long));
        if (e == hipSuccess) e = hipMemsetAsync(stamps, 0, nst * sizeof(long long), s);
        if (e == hipSuccess) e = hipMemcpyToSymbolAsync(HIP_SYMBOL(g_pp_stamps), &stamps, sizeof stamps, 0,
                                                        hipMemcpyHostToDevice, s);
        if (e != hipSuccess) return e;
    }
    const bool fold = interp || !in;
#define PAMG_FPP1(TS, NT, RB_, K_, F_)                                                                                     \
    hipLaunchKernelGGL((k_face_pp<TS, NT, RB_, K_, F_>), g, dim3(NT), 0, s, in, out_pre, out_mid, out_end, out_end2, L.RHS, \
                       L.stc,                                                                                            \
                       L.fnb, L.fface, L.fsx, L.gtab, L.gpat, P.d_hface, P.d_bcv, L.cpos, L.cnb, L.nup, L.pitch, l1, rdt, res,  \
                       R, RC, pc, TC)
#define PAMG_FPP(TS, NT, RB_, K_) \
    do { if (fold) PAMG_FPP1(TS, NT, RB_, K_, true); else PAMG_FPP1(TS, NT, RB_, K_, false); } while (0)
#define PAMG_FPPK(TS, NT)                                          \
    if (rb) { if (K == 2) PAMG_FPP(TS, NT, true, 2); else PAMG_FPP(TS, NT, true, 1); } \
    else { if (K == 2) PAMG_FPP(TS, NT, false, 2); else PAMG_FPP(TS, NT, false, 1); }
    if (L.nsub == 256 && rb) {   // 136 ups: 192 threads, one each
        if (K == 2) PAMG_FPP(256, 192, true, 2); else PAMG_FPP(256, 192, true, 1);
    } else if (L.nsub == 1024) { PAMG_FPPK(1024, 512) }
    else if (L.nsub == 256) { PAMG_FPPK(256, 128) }
    else return hipErrorInvalidValue;   // (4,096: the iterate and RHS exceed the LDS)
#undef PAMG_FPPK
#undef PAMG_FPP
#undef PAMG_FPP1
    hipError_t e = hipGetLastError();
    if (stamp_path) {
        std::vector<long long> hst(nst);
        long long *null = nullptr;
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (e == hipSuccess) e = hipMemcpy(hst.data(), stamps, nst * sizeof(long long), hipMemcpyDeviceToHost);
        if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(g_pp_stamps), &null, sizeof null);
        (void)hipFree(stamps);
        if (FILE *f = fopen(stamp_path, "ab")) {
            const long long hdr[4] = {(long long)g.x, kPPStamps, L.nsub, K};
            fwrite(hdr, sizeof hdr, 1, f);
            fwrite(hst.data(), sizeof(long long), nst, f);
            fclose(f);
        }
    }
    return e;
}

int face_chain_per_wg(int nsub, int U, int cus) {
    const int g = std::max(1, std::min(cus, U));
    const int k = (U + g - 1) / g;
    return (int)std::min<int64_t>((int64_t)k * nsub, 1 << 30);
}

bool face_chain_fits(int nsub, int U, int cus) {
    const int E = face_chain_per_wg(nsub, U, cus);
    int m = 1;
    while (m * m < nsub) m *= 2;
    return U >= 1 && E <= kChainNT * kChainPer && 9 * (E / nsub) * m <= kChainHalo;
}

hipError_t launch_face_chain(hipStream_t s, const Level &L, int U, int cus, double *tov, double *tov_b, double *tovo,
                             unsigned *flags, const int *nb_off, const int *nb_list, unsigned *tmo, int run, int total,
                             int store, bool rb, bool level1, double rdt, double omega, int slots, bool from_T,
                             unsigned f0, int guard, ChainGate G) {
    if (L.N == 0 || run <= 0) return hipSuccess;
    if (G.gate && (!guard || !G.stat)) return hipErrorInvalidValue;   // the gate reports the guard's outcome
    // store 1: tnew := the iterate before the last sweep, tnew_nonlin := the last; 2: tnew := the last (a dead
    // last sweep); 3: both := the last (the corrected cycle's coarsest call, tnew := tnew_nonlin after it)
    if (!face_chain_fits(L.nsub, U, cus) || !L.fnb || store < 1 || store > 3) return hipErrorInvalidValue;
    const int g = std::max(1, std::min(cus, U));
    const int k = (U + g - 1) / g;
    const int grid = (U + k - 1) / k;
    const int E = k * L.nsub;
    const HaloPlan &P = L.halo;
    HaloArgs H{P.d_hsub, P.d_hface, P.d_bcv, P.d_told_halo, tov, tovo, P.d_send, 1 << L.isplit};
    int lg = log2i(L.nsub), l1 = level1 ? 1 : 0;
    double *T = L.T, *TNN = L.TNN;
    const double *RHS = L.RHS, *stc = L.stc, *fface = L.fface;
    const int4 *fnb = L.fnb;
    const int *fsx = L.fsx;
    int64_t pitch = L.pitch, N = L.N;
    // PAMG_CHAIN_STAMPS=<file> (a PAMG_STAMPS=1 diagnostics build): append every launch's per-sweep phase stamps
    // of workgroups 0..7
    static const char *stamp_path = PAMG_STAMPS ? getenv("PAMG_CHAIN_STAMPS") : nullptr;
    long long *stamps = nullptr;
    // the per-wave chain stamps every wave of workgroups 0..7 (kPWStamps a sweep), the workgroup chain
    // thread 0 of each (4 a sweep); the header's sign tells them apart
    const size_t nst_pw = (size_t)8 * kPW * run * kPWStamps;
    const size_t nst = std::max((size_t)8 * run * 4, nst_pw);
    if (stamp_path) {
        hipError_t e = hipMalloc(&stamps, nst * sizeof(long long));
        if (e != hipSuccess) return e;
        e = hipMemsetAsync(stamps, 0, nst * sizeof(long long), s);
        if (e != hipSuccess) return e;
    }
    const int *cpos = L.cpos;
    int nup = L.nup;
    const double *SRC = from_T ? L.T : L.TNN;
    // the publish point (k_face_chain): 3 the words and the flag right after the up pass, which is split around
    // the wait; 2 the same without the split; 0 after the down pass (a level whose words are not all on up
    // sub-elements). Measured: 0 -> 2 -> 3, 10.4 -> 9.1 -> 8.7 us per sweep (profiles/r03_n_face_chain_early.txt)
    int nui = L.nui, early = L.words_up ? 3 : 0;
    // the split up pass needs each half's items in one item per thread
    if (early == 3 && !(nui > 0 && (int64_t)k * nui <= kChainNT && (int64_t)k * (L.nup - nui) <= kChainNT)) early = 2;
    // PAMG_CHAIN_SNAP16=0: the snapshot's 8-byte loads, the form a snapshot buffer beyond a buffer
    // resource's 32-bit range takes (read per launch: a test switches it within a process)
    const char *snap_env = getenv("PAMG_CHAIN_SNAP16");
    int snap_ok = !(snap_env && atoi(snap_env) == 0);
    void *args[] = {&T, &TNN, &SRC, &RHS, &stc, &fnb, &fface, &fsx, &tov, &tov_b, &H, &flags, &nb_off, &nb_list, &tmo,
                    &run, &total, &store, (void *)&E, &pitch, &N, &lg, &slots, &l1, &rdt, &omega, &cpos, &nup, &nui, &early, &f0,
                    &snap_ok, &stamps, &guard, &G};
    // the LDS records and item lists need the colour lists' sizes to fit the items (KU = 2, KD = 1)
    const bool uni = L.nsub >= 64,
               lrec = k <= kChainRec && L.cpos && (int64_t)k * L.nup <= 2 * kChainNT && (int64_t)k * L.ndn <= kChainNT;

#define PAMG_CHF(U_, R_) (lrec ? (const void *)k_face_chain<U_, R_, true> : (const void *)k_face_chain<U_, R_, false>)
    const void *f = uni ? (rb ? PAMG_CHF(true, true) : PAMG_CHF(true, false))
                        : (rb ? PAMG_CHF(false, true) : PAMG_CHF(false, false));
#undef PAMG_CHF
    // the per-wave form (k_face_chain_pw): red-black with the split up pass, whole un_eles per wave whose
    // colour lists fit 64 lanes, per-wave flags (face_chain_setup sizes them); PAMG_CHAIN_PW=0 keeps the
    // workgroup form (read per launch: a test switches it within a process)
    const char *pw_env = getenv("PAMG_CHAIN_PW");
    const int qpw = (k + kPW - 1) / kPW;
    if (!(pw_env && atoi(pw_env) == 0) && rb && lrec && early == 3 && uni && L.nsub <= 64 &&
        qpw * std::max(nui, std::max(L.nup - nui, L.ndn)) <= 64)
        f = (const void *)k_face_chain_pw;
    // the per-wave chain's flags: one per workgroup, stored by its last wave to publish, and one polling wave per
    // workgroup (bits 32 and 64; one flag per wave measured slower: profiles/r05_y_chain_wgflag.txt,
    // r05_z_chain_leader_poll.txt)
    if (f == (const void *)k_face_chain_pw) early |= 32 | 64;
    hipError_t e = launch_coresident(f, grid, kChainNT, args, s);
    if (stamp_path) {
        std::vector<long long> h(nst);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (e == hipSuccess) e = hipMemcpy(h.data(), stamps, nst * sizeof(long long), hipMemcpyDeviceToHost);
        (void)hipFree(stamps);
        if (FILE *fp = fopen(stamp_path, "ab")) {
            const bool pw = f == (const void *)k_face_chain_pw;
            const long long hdr[4] = {pw ? -run : run, grid, E, L.nsub};
            fwrite(hdr, sizeof hdr, 1, fp);
            fwrite(h.data(), sizeof(long long), pw ? nst_pw : (size_t)8 * run * 4, fp);
            fclose(fp);
        }
    }
    return e;
}

// the wavefront call (k_face_wave): levels whose un_eles are 256, 1,024 or 4,096 sub-elements
bool face_wave_shape(const Level &L) {
    const int m = L.nsub == 256 ? 16 : L.nsub == 1024 ? 32 : L.nsub == 4096 ? 64 : 0;
    // the colour lists' sizes are the kernel's compile-time item counts
    return m && L.N % L.nsub == 0 && L.cpos && L.nup == m * (m + 1) / 2;
}

namespace {
const void *face_wave_fn(int nsub, bool rb, int *nt) {
    switch (nsub) {
        case 4096: *nt = 1024; return rb ? (const void *)k_face_wave<4096, 1024, true> : (const void *)k_face_wave<4096, 1024, false>;
        case 1024: *nt = 256; return rb ? (const void *)k_face_wave<1024, 256, true> : (const void *)k_face_wave<1024, 256, false>;
        case 256: *nt = 64; return rb ? (const void *)k_face_wave<256, 64, true> : (const void *)k_face_wave<256, 64, false>;
        default: *nt = 0; return nullptr;
    }
}
}  // namespace

// co-resident workgroups of the wavefront kernel for this level (0: not launchable)
int face_wave_grid(const Level &L, bool rb, int cus) {
    int nt = 0, per = 0;
    const void *f = face_wave_fn(L.nsub, rb, &nt);
    if (!f || hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, f, nt, 0) != hipSuccess) return 0;
    return per * cus;
}

hipError_t launch_face_wave(hipStream_t s, const Level &L, int U, int grid, double *tov, double *tov_b, double *tovo,
                            unsigned long long *g0, unsigned long long *g1, unsigned tag0, unsigned *flags,
                            const int *order, unsigned *tmo, int run, int total, int store, bool rb, bool level1,
                            double rdt, int slots, bool from_T) {
    if (L.N == 0 || run <= 0) return hipSuccess;
    int nt = 0;
    const void *f = face_wave_fn(L.nsub, rb, &nt);
    if (!f || !face_wave_shape(L) || !L.fnb || grid <= 0) return hipErrorInvalidValue;
    const HaloPlan &P = L.halo;
    HaloArgs H{P.d_hsub, P.d_hface, P.d_bcv, P.d_told_halo, tov, tovo, P.d_send, 1 << L.isplit};
    int l1 = level1 ? 1 : 0;
    double *T = L.T, *TNN = L.TNN;
    const double *RHS = L.RHS, *stc = L.stc, *fface = L.fface;
    const int4 *fnb = L.fnb;
    const int *fsx = L.fsx;
    int64_t pitch = L.pitch;
    hipError_t e = hipMemsetAsync(flags, 0, sizeof(unsigned) * ((size_t)U + 1), s);
    if (e != hipSuccess) return e;
    // PAMG_WAVE_STAMPS=<file>: append every launch's per-ticket phase stamps of workgroups 0..7
    static const char *stamp_path = PAMG_STAMPS ? getenv("PAMG_WAVE_STAMPS") : nullptr;   // (diagnostics build)
    long long *stamps = nullptr;
    const size_t nst = (size_t)8 * kWaveStampT * kWaveStampW;
    if (stamp_path) {
        e = hipMalloc(&stamps, nst * sizeof(long long));
        if (e != hipSuccess) return e;
        e = hipMemsetAsync(stamps, 0, nst * sizeof(long long), s);
        if (e != hipSuccess) return e;
    }
    const int g = std::min(grid, U);
    const int *cpos = L.cpos;
    int nup = L.nup;
    const double *SRC = from_T ? L.T : L.TNN;
    void *args[] = {&T, &TNN, &SRC, &RHS, &stc, &fnb, &fface, &fsx, &cpos, &nup, &tov, &tov_b, &g0, &g1, &tag0, &H, &flags,
                    &order, &tmo, &U, &run, &total, &store, &pitch, &slots, &l1, &rdt, &stamps};
    e = launch_coresident(f, g, nt, args, s);
    if (stamp_path) {
        std::vector<long long> hs(nst);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (e == hipSuccess) e = hipMemcpy(hs.data(), stamps, nst * sizeof(long long), hipMemcpyDeviceToHost);
        (void)hipFree(stamps);
        if (FILE *fp = fopen(stamp_path, "ab")) {
            const long long hdr[4] = {run, g, U, L.nsub};
            fwrite(hdr, sizeof hdr, 1, fp);
            fwrite(hs.data(), sizeof(long long), nst, fp);
            fclose(fp);
        }
    }
    return e;
}

hipError_t launch_face_residual(hipStream_t s, const Level &L, const double *tov, bool neg, bool level1, double rdt,
                                int slots) {
    if (L.N == 0) return hipSuccess;
    if (!L.fnb || !L.fface || !L.fsx) return hipErrorInvalidValue;
    const dim3 g(grid_for(L.N)), b(kBlock);
    const int lg = log2i(L.nsub), l1 = level1 ? 1 : 0;
    const bool uni = L.nsub >= 64;
    const double omega = 0.0;
    if (neg) {
        PAMG_FACE(4, L.T, L.RES);
    } else {
        PAMG_FACE(3, L.T, L.RES);
    }
#undef PAMG_FACE
    return hipGetLastError();
}

}  // namespace pamg
