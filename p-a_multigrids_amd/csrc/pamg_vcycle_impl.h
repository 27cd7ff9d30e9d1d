// Fused V-cycle for gfx950: two launches run one pass of the n_multigrid
// loop body of transport_tri_semi.F90:319-379 for every un_ele.
//
// Every operation of the V-cycle is local to one unstructured element (the
// smoother, residual and RHS use the element's 3x3 operator; the children of a
// coarse sub-element live in the same un_ele, splitting.F90:97-140), so a
// workgroup carries a tile of whole un_eles through its part of the cycle
// without exchanging data with other workgroups. The computation is the
// reference's, step for step and in its operation order (same device helpers
// as the per-step kernels; the state after every cycle is bitwise equal to
// pamg_vcycle's multi-kernel form, tests/test_gpu_parity.py). The schedule
// follows the data dependences, which the block-diagonal operator leaves loose:
//   * the restrictor (:336) reads the residual of the PREVIOUS cycle, so it is
//     evaluated where that residual is produced and kept as RHSN (the next
//     cycle's RHS) -- no launch re-reads a residual;
//   * the prolongation-leg smoother of level l (:376) starts from
//     tnew_nonlin = the restriction-leg tnew of level l (:367); the prolonged
//     values are overwritten at its first sweep (:550), so every level's two
//     smoother calls depend on its own state only;
//   * the halo words (update_overlaps, :555) have no reader in the cycle; the
//     last writer of every word is level 1's prolongation-leg smoother call
//     (the coarser levels write subsets of its slots), so the cycle writes each
//     word once, with that value (t_overlap_old and the boundary words, which
//     do not change within a time step: k_overlap_static, once per step).
// Launch 1, k_vc_coarse: levels 2..L -- one wave per tile, the lane's share of
//   every level in registers, the levels smoothed in lockstep (the coarsest
//   level's 1 + 15 smoother calls are a chain of dependent sweeps; the other
//   levels' calls are interleaved into it), the prolongator cascades among them.
// Launch 2, k_vc_fine: level 1 -- both smoother calls, get_residual, the
//   restrictor of its residual into level 2's RHSN, and the prolongator cascade
//   from the final level-2 tnew; a streaming kernel (tnew, RHS in; residual,
//   tnew, tnew_nonlin out).
// The pipelined form runs level 1 of cycle c and the coarse levels of cycle c+1 in
// one launch (k_vc_fine<.., PIPE>); the resident form (k_vc_res, k_vc_resb, the
// default) runs every cycle of a pamg_vcycle call in one launch with the tiles'
// state on-chip between cycles.
// Levels are 0-based inside this file: level 0 = the reference's level 1.
//
// (pamg_vcycle_impl.h: the kernels and their launch templates, instantiated per n_split in
// pamg_vcycle_s.hip -- one translation unit per n_split, compiled in parallel -- and dispatched
// by pamg_vcycle.hip)
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <cstdio>
#include <algorithm>
#include <cstdlib>
#include <type_traits>
#include <vector>

#include "pamg_device.h"
#include "pamg_internal.h"

namespace pamg {
// the launch arguments, shared by the per-n_split translation units and the dispatcher
namespace vc {
using detail::HaloArgs;
// the planes of a level are one allocation (pamg_api.cpp): tnew, tnew_nonlin, RHS,
// residual, told, RHSN at plane offsets 0, 3, 6, 9, 12, 15 (one base pointer in SGPRs)
struct VLevel {
    double *base;
    __device__ __forceinline__ double *T() const { return base; }
    __device__ __forceinline__ double *TNN() const { return base + 3 * pitch; }
    __device__ __forceinline__ double *RHS() const { return base + 6 * pitch; }
    __device__ __forceinline__ double *RES() const { return base + 9 * pitch; }
    __device__ __forceinline__ double *TOLD() const { return base + 12 * pitch; }
    __device__ __forceinline__ double *RHSN() const { return base + 15 * pitch; }
    __device__ __forceinline__ double *SRC() const { return base + 18 * pitch; }   // level 0 only
    const double *stc;
    int64_t pitch;
    HaloArgs H;
};

struct VArgs {
    VLevel lv[kMaxFusedLevels];
    int64_t U;
    int n_smooth, n_coarse;
    double rdt;
    double *rhsn2;          // level 2's RHSN buffer: read by the coarse launch, written by the level-1 launch
    long long *stamps;      // phase timeline (PAMG_VCYCLE_STAMPS diagnostics), null otherwise
    int keep;               // the dead-until-final stores the launch makes (kKeep*)
    int64_t tile0;          // first tile of the launch (a launch may cover a range of tiles)
    // RHSF launches (the first of a pamg_run step, told := tnew and level 1's RHS from it) with
    // kKeepTold: the second send buffer, whose told halves it writes too
    double *send_b;
    int cycles;             // the resident launch: cycles of the call (of each time step)
    int steps;              // the resident launch starting time steps (RHSF): steps of the run, each
                            // told := tnew and its RHS, then `cycles` cycles; 1 otherwise
    // the resident launch with an exchange after every cycle (part 6, halo_exchange = 1): cycle c <
    // cycles - 1 packs the tnew words of its remote halo entries into ring + c ring_stride (3 per
    // entry); each workgroup counts the cycle in xc_done[c] and the one that completes it adds 1 to
    // *xc_sig, the signal the comm stream waits on (pamg_api.cpp vcycle_fused)
    double *ring;
    int64_t ring_stride;
    unsigned *xc_done;
    unsigned long long *xc_sig;
    unsigned xc_grid;
    // the resident call with its per-call exchange started early (pamg_api.cpp vcycle_fused): tile_map
    // (non-null) gives workgroup b the tile tile_map[b] -- the tiles holding a face whose neighbour is on
    // another rank first, so that they finish in the first round; each such tile counts its end in
    // *xe_done after its last cycle's send words are drained (written through), and the one whose count
    // reaches xe_n (the running total, the counter is never reset) adds 1 to *xc_sig: the comm stream's
    // signal to exchange while the other tiles run
    const int *tile_map;
    unsigned *xe_done;
    unsigned xe_n;
};

}  // namespace vc

namespace {
using vc::VArgs;
using vc::VLevel;

using namespace detail;

// level-1 launch: a tile of 2**TL level-0 sub-elements (whole un_eles, TL >= 2 n_split) on
// 2**(TL-1) threads, one adjacent pair each. TL = max(2 n_split, PAMG_FINE_TL_MIN) = 10: 1024
// sub-elements, 512 threads (one un_ele at n_split = 5). Measured (scripts/ab2.sh): 256-element
// tiles (PAMG_FINE_TL_MIN=8, 4x the workgroups at n_split <= 4) are 7-9 % slower at n_split = 3
// and 4. Occupancy: the kernel wants 71 VGPRs (7 waves per SIMD, 3 workgroups per CU); bounded
// to 64 (W8: 8 waves, 4 workgroups per CU) it is 0.8 % slower on a full mesh but fits 1,024
// workgroups -- a rank's share of untitled8192 on 8 GPUs -- in one round instead of two
// (0.0350 -> 0.0312 ms per cycle, scripts/ab_strong.sh): see launch_slt.
#ifndef PAMG_FINE_TL_MIN
#define PAMG_FINE_TL_MIN 10
#endif
// level-1 tnew loads / stores and RHS loads of the V-cycle launches (A/B builds)
#ifndef PAMG_NT_TL
#define PAMG_NT_TL ((PAMG_NT & 1) != 0)
#endif
#ifndef PAMG_NT_TS
#define PAMG_NT_TS ((PAMG_NT & 2) != 0)
#endif
#ifndef PAMG_NT_RL
#define PAMG_NT_RL ((PAMG_NT & 1) != 0)
#endif
// issue priority of the pipelined launch's coarse tail (A/B builds; 1 and 2 measured within noise
// of 0, profiles/r01_v18_tail_prio_ab.txt)
#ifndef PAMG_TAIL_PRIO
#define PAMG_TAIL_PRIO 0
#endif
#ifndef PAMG_CHAIN_PRIO
#define PAMG_CHAIN_PRIO 3
#endif
// at n_split >= 6 a tile is a part of one un_ele (2**(2 n_split - 10) tiles each): the storage
// order (pamg_internal.h Level::pos) gives every aligned block of 4**k level-1 sub-elements its
// own coarser sub-elements, so a tile never needs another's data at any level
constexpr int kFineTLMax = 10;
constexpr int fine_tl(int S) {
    return (2 * S < kFineTLMax ? 2 * S : kFineTLMax) > PAMG_FINE_TL_MIN ? (2 * S < kFineTLMax ? 2 * S : kFineTLMax)
                                                                        : PAMG_FINE_TL_MIN;
}
// level-0 sub-elements per thread: an adjacent pair (16-byte accesses); one at n_split <=
// PAMG_NP1_MAX_S (A/B builds: twice the waves for the single-round launches of small n_split).
// Measured (scripts/ab2.sh, parity-tested): equal at n_split = 2 and 3 (those launches stream
// at ~5.3 TB/s plus ~2.8 us of launch overhead, scripts/micro/launch.hip), 37 % slower at
// n_split = 4, L = 4 -- the pair stays everywhere
#ifndef PAMG_NP1_MAX_S
#define PAMG_NP1_MAX_S 0
#endif
constexpr int fine_np(int S) { return S <= PAMG_NP1_MAX_S ? 1 : 2; }
constexpr int fine_mt(int S) { return (1 << fine_tl(S)) / fine_np(S); }
constexpr int kMTc = 64;    // threads per workgroup, coarse-level kernel (one wave per tile)

// Stores of a pipelined launch whose values the rest of the call overwrites before any read
// ("final-cycle stores"): level 1's residual and tnew_nonlin (the next launch
// rewrites both; the residual's one reader, the restrictor, takes it from LDS here), the
// coarse levels' RHS and residual (rewritten by the next launch's coarse part; read from
// registers and LDS in this one) and the halo words (rewritten every cycle; exchanged after
// the call's last cycle with halo_exchange = 0). The call's final level-1 launch (k_vc_fine,
// PIPE = false) stores all of level 1's fields and halo words; its last pipelined launch, the
// one that leaves the coarse levels at their final cycle, keeps kKeepCoarse. Inside pamg_run
// every step but the last skips those too (the next step overwrites them unread).
constexpr int kKeepL1 = PAMG_KEEP_L1, kKeepCoarse = PAMG_KEEP_COARSE, kKeepHalo = PAMG_KEEP_HALO;
constexpr int kKeepTold = PAMG_KEEP_TOLD;

// phase stamps: 100 MHz wall clock per wave at the phase boundaries, plus the wave's HW_ID
// (diagnostics build only: make PAMG_STAMPS=1; the pointer costs SGPRs the kernels need)
#ifndef PAMG_STAMPS
#define PAMG_STAMPS 0
#endif
constexpr int kStampSlots = 10;
template <int MT>
__device__ __forceinline__ void stamp(const VArgs &A, int i) {
    if (PAMG_STAMPS && A.stamps && (threadIdx.x & 63) == 0)
        A.stamps[((int64_t)blockIdx.x * (MT / 64) + (threadIdx.x >> 6)) * kStampSlots + i] = wall_clock64();
}
template <int MT>
__device__ __forceinline__ void stamp_hwid(const VArgs &A) {
    if (PAMG_STAMPS && A.stamps && (threadIdx.x & 63) == 0) {
        unsigned hw;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        A.stamps[((int64_t)blockIdx.x * (MT / 64) + (threadIdx.x >> 6)) * kStampSlots + 9] = hw;
    }
}

// tile geometry (0-based level l): 4**(S-l) sub-elements per un_ele; a tile holds
// T >> 2l sub-elements of level l (T / 4**S un_eles, or a part of one), T = 2**TL. Tile b
// covers the global indices b nt(l) .. (b + 1) nt(l) - 1 of every level l (the storage order
// puts the children of global g at 4g .. 4g+3, Level::pos); an index is valid below
// N_l = U 4**(S-l) (the last tile of a mesh whose U is not a multiple of its un_eles).
template <int S, int L>
struct Geo {
    static constexpr int C = L - 1;                                // coarsest level
    static constexpr int TL = fine_tl(S);
    static constexpr int T = 1 << TL;                              // level-0 sub-elements per tile
    static constexpr int NP = fine_np(S);                          // level-0 sub-elements per thread
    static constexpr int MT = T / NP;                              // threads of the level-1 launch
    static constexpr int lg(int l) { return 2 * (S - l); }
    static constexpr int nt(int l) { return T >> (2 * l); }
    // each wave inside one un_ele (a wave spans 64 NP level-0 sub-elements, 64 of any other level)
    static constexpr bool uni(int l) { return lg(l) >= (l == 0 ? (NP == 2 ? 7 : 6) : 6); }
};

// tile b of level l: global index of its local sub-element i (valid: below N_l = U 4**(S-l);
// invalid ones are clamped to the tile's first index, so loads stay in bounds)
template <int S>
__device__ __forceinline__ uint32_t tile_index(const VArgs &A, int64_t b, int ntl, int l, int i, bool &valid) {
    const uint32_t g0 = (uint32_t)(b * ntl), n = (uint32_t)(A.U << (2 * (S - l)));
    valid = i < ntl && g0 + (uint32_t)i < n;
    return g0 + (uint32_t)(valid ? i : 0);
}

// field access: wave-uniform plane base (SGPRs) + 32-bit sub-element index (one VGPR for all planes)
// 8-byte accesses stay plain: non-temporal 8-B lanes measured 15 % slower on the pipelined
// launch (their lines are not merged in L1)
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
// streamed with non-temporal 16-byte loads and stores (pamg_device.h PAMG_NT)
typedef double v2d __attribute__((ext_vector_type(2)));
template <bool NT = (PAMG_NT & 1) != 0>
__device__ __forceinline__ void load3p(const double *f, int64_t pitch, uint32_t s, double a[3], double b[3]) {
    const uint32_t o = s << 3;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        const v2d *q = reinterpret_cast<const v2d *>(reinterpret_cast<const char *>(f + c * pitch) + o);
        const v2d v = NT ? __builtin_nontemporal_load(q) : *q;
        a[c] = v.x;
        b[c] = v.y;
    }
}
template <bool NT = (PAMG_NT & 2) != 0>
__device__ __forceinline__ void store3p(double *f, int64_t pitch, uint32_t s, const double a[3], const double b[3]) {
    const uint32_t o = s << 3;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        v2d *q = reinterpret_cast<v2d *>(reinterpret_cast<char *>(f + c * pitch) + o);
        const v2d v = {a[c], b[c]};
        if (NT) __builtin_nontemporal_store(v, q);
        else *q = v;
    }
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
template <class ST>
__device__ __forceinline__ void stencil(bool uni, const double *__restrict__ stc, uint32_t u, ST &S) {
    if (uni) u = __builtin_amdgcn_readfirstlane(u);
    load_stc(stc + u * (uint32_t)kStcStride, S);
}

// n sweeps of one smoother call (n_smooth, :491-507): x the last iterate (tnew_nonlin), p the
// one before it (tnew, :550 vs :693) -- copied once, before the last sweep (p unchanged if n = 0)
template <class ST>
__device__ __forceinline__ void sweeps1(const ST &S, double rdt, int n, const double b[3], double x[3], double p[3]) {
    if (n <= 0) return;
    for (int it = 1; it < n; ++it) sweep(S, rdt, b, x);
    copy3(p, x);
    sweep(S, rdt, b, x);
}

// one smoother call inside a fused cycle when only its tnew is read: the iterate before the last
// sweep (:550 vs :693); the last sweep feeds only a tnew_nonlin the cycle overwrites unread
// (dead computation), so the call is n - 1 sweeps in place (N sub-elements, interleaved)
template <int N, class ST>
__device__ __forceinline__ void sweeps_tnew(const ST &S, double rdt, int n, const double b[N][3], double x[N][3]) {
    for (int it = 1; it < n; ++it) {
#pragma unroll
        for (int q = 0; q < N; ++q) sweep(S, rdt, b[q], x[q]);
    }
}

// two sub-elements of one un_ele, interleaved
template <class ST>
__device__ __forceinline__ void sweeps2(const ST &S, double rdt, int n, const double b0[3], const double b1[3],
                                        double x0[3], double x1[3], double p0[3], double p1[3]) {
    if (n <= 0) return;
    for (int it = 1; it < n; ++it) {
        sweep(S, rdt, b0, x0);
        sweep(S, rdt, b1, x1);
    }
    copy3(p0, x0);
    copy3(p1, x1);
    sweep(S, rdt, b0, x0);
    sweep(S, rdt, b1, x1);
}

// N sub-elements of one un_ele, interleaved
template <int N, class ST>
__device__ __forceinline__ void sweepsN(const ST &S, double rdt, int n, const double b[N][3], double x[N][3],
                                        double p[N][3]) {
    if (n <= 0) return;
    for (int it = 1; it < n; ++it) {
#pragma unroll
        for (int q = 0; q < N; ++q) sweep(S, rdt, b[q], x[q]);
    }
#pragma unroll
    for (int q = 0; q < N; ++q) copy3(p[q], x[q]);
#pragma unroll
    for (int q = 0; q < N; ++q) sweep(S, rdt, b[q], x[q]);
}

template <class ST>
__device__ __forceinline__ void residual(const ST &S, double rdt, const double p[3], const double b[3], double r[3]) {
    resid(S, rdt, p, b, r);
}

// ---- halo words of one sub-element (update_overlaps, :555)
// h: its positions along faces 1..3 packed 10 bits each (0: not on that face; 2**i_split <= 256)
__device__ __forceinline__ int hs_pack(int4 q) { return q.x | (q.y << 10) | (q.z << 20); }

// tnew words of the halo (update_overlaps); t_overlap_old and the boundary values are
// constant within a time step and are written by k_overlap_static (pamg_kernels.hip)
__device__ __forceinline__ void hs_write(bool uni, const HaloArgs &H, uint32_t u, int h, const double t[3]) {
    if (h == 0) return;
    if (uni) u = __builtin_amdgcn_readfirstlane(u);
    const int4 r1 = H.hface[3 * u], r2 = H.hface[3 * u + 1], r3 = H.hface[3 * u + 2];
    const int a = h & 1023, b = (h >> 10) & 1023, c = h >> 20;
    // the send words written through: the early exchange may read them while the launch runs
    if (a) halo_face<true, false, false, true>(H, r1, 1, a, t, t);
    if (b) halo_face<true, false, false, true>(H, r2, 2, b, t, t);
    if (c) halo_face<true, false, false, true>(H, r3, 3, c, t, t);
}

// the tnew words of one sub-element's remote halo entries (mode 2) into a ring buffer of 3 words
// per entry (the per-cycle exchange of the resident call), written through (sc1: the hand-off form
// of cdna_hip_programming.md 6 Guideline 16 R1, no release fence)
__device__ __forceinline__ void hs_ring(bool uni, const HaloArgs &H, double *ring, uint32_t u, int h,
                                        const double t[3]) {
    if (h == 0) return;
    if (uni) u = __builtin_amdgcn_readfirstlane(u);
    const int pos[3] = {h & 1023, (h >> 10) & 1023, h >> 20};
#pragma unroll
    for (int f = 0; f < 3; ++f) {
        if (!pos[f]) continue;
        const int4 r = H.hface[3 * u + f];
        if ((r.x & 3) != 2) continue;
        double *o = ring + 3 * (int64_t)(r.z + pos[f] - 1);
#pragma unroll
        for (int c = 0; c < 3; ++c) st_coh(o + c, t[c]);
    }
}

// a workgroup's end of cycle c (after the barrier that follows every wave's drained write-through
// ring stores): count it with a relaxed agent-scope add; the workgroup whose add completes the cycle
// publishes it to the comm stream's signal. The ring words are already at the coherence point (sc1,
// drained), so neither add needs a fence: an acq_rel add here cost a buffer_wbl2 + buffer_inv per
// workgroup and cycle (halo_exchange = 1 ran at 0.39 of the plain call, profiles/r03_a_mp_detached_*)
__device__ __forceinline__ void xc_signal(const VArgs &A, int c) {
    const unsigned old = __hip_atomic_fetch_add(A.xc_done + c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (old + 1 == A.xc_grid) __hip_atomic_fetch_add(A.xc_sig, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// a remote tile's end of the call (after the barrier that follows its waves' drained write-through
// send words): the count that completes the remote tiles raises the comm stream's signal (the form of
// xc_signal, once per call)
__device__ __forceinline__ void xe_signal(const VArgs &A) {
    const unsigned old = __hip_atomic_fetch_add(A.xe_done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (old + 1 == A.xe_n) __hip_atomic_fetch_add(A.xc_sig, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// the tile of this workgroup: the early exchange's order (remote tiles first), else the grid's
__device__ __forceinline__ int64_t resident_tile(const VArgs &A) {
    return A.tile_map ? (int64_t)A.tile_map[blockIdx.x] : (int64_t)blockIdx.x + A.tile0;
}

// XC: does tile tb (T level-1 sub-elements from tb T) hold a face whose neighbour is on another rank?
// Only such a tile stores ring words, so only its waves drain them before the cycle's count (an
// x-strip rank of untitled8192 at N = 2: 64 of 4,096 tiles); the others count without waiting
template <int S, int T>
__device__ __forceinline__ bool tile_remote(const VArgs &A, int64_t tb) {
    int64_t u0 = (tb * T) >> (2 * S), u1 = ((tb + 1) * T - 1) >> (2 * S);
    if (u1 >= A.U) u1 = A.U - 1;
    bool r = false;
    for (int64_t u = u0; u <= u1; ++u)
#pragma unroll
        for (int f = 0; f < 3; ++f) r |= (A.lv[0].H.hface[3 * u + f].x & 3) == 2;
    return r;
}

// the words of one sub-element that are constant within a time step (k_overlap_static's, from
// its told `to`): t_overlap_old of the neighbour, the boundary values of both arrays, the told
// half of a send entry -- into both send buffers -- and the compact told copy of the halo
__device__ __forceinline__ void hs_write_static(const HaloArgs &H, double *send_b, uint32_t u, int h,
                                                const double to[3]) {
    if (h == 0) return;
    const int pos[3] = {h & 1023, (h >> 10) & 1023, h >> 20};
#pragma unroll
    for (int f = 0; f < 3; ++f) {
        if (!pos[f]) continue;
        const int4 r = H.hface[3 * u + f];
        halo_face<false, true>(H, r, f + 1, pos[f], to, to);
        const int mode = r.x & 3;
        if (mode == 0) continue;
        double *o = const_cast<double *>(H.told) + 3 * (int64_t)(r.w + pos[f] - 1);
#pragma unroll
        for (int c = 0; c < 3; ++c) o[c] = to[c];
        if (mode == 2 && send_b) {
            double *q = send_b + 6 * (int64_t)(r.z + pos[f] - 1);
#pragma unroll
            for (int c = 0; c < 3; ++c) q[3 + c] = to[c];
        }
    }
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
// level 1, one of level 2, one on the first nt(l) lanes below. The lane's share of
// every coarse level -- a "chunk" per (level, k) -- lives in registers for the whole
// cycle, and the levels are smoothed in lockstep: the data dependences of the cycle
//  tie a level's smoother calls to its own earlier ones and to the
// prologue only (the restrictor reads the PREVIOUS cycle's residual), so
//   phase A: the restriction-leg smoother call of every level, interleaved, then
//            get_residual of every level;
//   phase B: the 1 + n_coarse smoother calls of the coarsest level, with the
//            prolongation-leg call of every other level interleaved into its first
//            n_smooth sweeps.
// A sweep is a chain of 8 dependent fp64 operations; interleaving the chunks keeps
// the wave issuing instead of waiting on that latency.
template <int S, int L>
struct CGeo {
    using G = Geo<S, L>;
    static constexpr int C = G::C;
    // tile: 2**TL level-1 sub-elements (the reference's finest level): one un_ele at n_split = 5,
    // a quarter of one at 6 (and so on), at least 256 level-1 sub-elements below (enough waves for
    // the small meshes, whose un_eles then share a wave)
    static constexpr int TL = 2 * S > 8 ? (2 * S < kFineTLMax ? 2 * S : kFineTLMax) : 8;
    static constexpr int nt(int l) { return (1 << TL) >> (2 * l); }
    static constexpr int K(int l) { return nt(l) >= 64 ? nt(l) / 64 : 1; }
    // the lanes of a chunk inside one un_ele (operator record through the scalar cache)
    static constexpr bool uni(int l) { return (nt(l) < 64 ? nt(l) : 64) <= (1 << G::lg(l)); }
    // the whole level of the tile inside one un_ele: one operator record for all its chunks
    static constexpr bool one(int l) { return nt(l) <= (1 << G::lg(l)); }
    static constexpr int NCH = [] { int n = 0; for (int l = 1; l <= C; ++l) n += K(l); return n; }();
    static constexpr int lev(int j) { int l = 1; while (j >= K(l)) { j -= K(l); ++l; } return l; }
    static constexpr int kk(int j) { int l = 1; while (j >= K(l)) { j -= K(l); ++l; } return j; }
    // LDS images for the (dead) prolongator cascades: F_l (restriction-leg tnew, 1 <= l < C)
    // and Y_l (final tnew, 2 <= l <= C)
    static constexpr int F(int l) { int o = 0; for (int i = 1; i < l; ++i) o += 3 * nt(i); return o; }
    static constexpr int Y(int l) { int o = F(C); for (int i = 2; i < l; ++i) o += 3 * nt(i); return o; }
    // M_l (1 <= l < C): mean of the three new residual components of each sub-element,
    // the restrictor's input (splitting.F90:146-151)
    static constexpr int M(int l) { int o = Y(C + 1); for (int i = 1; i < l; ++i) o += nt(i); return o; }
    static constexpr int total = M(C) > 0 ? M(C) : 1;
};

template <int S, int L, class ST>
__global__ __launch_bounds__(kMTc, 3) void k_vc_coarse(VArgs A, const double *__restrict__ sp1,
                                                       const double *__restrict__ sp2, const double *__restrict__ sp3,
                                                       const double *__restrict__ sp4) {
    // operator records as restrict kernel arguments: never written here, so wave-uniform
    // records are fetched with scalar loads
    const double *__restrict__ SP[kMaxFusedLevels] = {nullptr, sp1, sp2, sp3, sp4};
    using G = Geo<S, L>;
    using Q = CGeo<S, L>;
    constexpr int C = G::C;
    constexpr int N = Q::NCH;
    static_assert(C >= 1, "coarse kernel needs two levels");
    __shared__ __attribute__((aligned(16))) double lds[Q::total];
    const int t = threadIdx.x;
    const double rdt = A.rdt;
    const int ns = A.n_smooth;
    const int64_t tb = (int64_t)blockIdx.x + A.tile0;   // tile
    stamp<kMTc>(A, 0);
    stamp_hwid<kMTc>(A);
    // chunk j = (level l, k): tile index t + 64 k; idle lanes (beyond the level or the
    // tile's un_eles) compute on index 0 and store nothing
    bool ok[N];
    uint32_t gx[N];
#pragma unroll
    for (int j = 0; j < N; ++j) {
        const int l = Q::lev(j), i = t + 64 * Q::kk(j);
        gx[j] = tile_index<S>(A, tb, Q::nt(l), l, i, ok[j]);
    }
    // operator records, fetched once: one per level when the tile's level lies in one un_ele
    // (scalar registers), else one per chunk (vector registers when the chunk spans un_eles)
    ST SL[C + 1], SC[N];
#pragma unroll
    for (int l = 1; l <= C; ++l)
        if (Q::one(l)) stencil(Q::uni(l), SP[l], (uint32_t)(tb * Q::nt(l)) >> G::lg(l), SL[l]);
#pragma unroll
    for (int j = 0; j < N; ++j)
        if (!Q::one(Q::lev(j))) stencil(Q::uni(Q::lev(j)), SP[Q::lev(j)], gx[j] >> G::lg(Q::lev(j)), SC[j]);
    auto stc_of = [&](int j, ST &St) { St = Q::one(Q::lev(j)) ? SL[Q::lev(j)] : SC[j]; };
    // ---- prologue: tnew of every level (tnew_nonlin := tnew, :327 / :348), halo positions,
    //      and the restrictor (:336) of every level: RHS_l := RHSN_l, the restriction of the
    //      PREVIOUS cycle's residual, computed when that residual was (below, and in the
    //      level-1 launch for level 1)
    double x[N][3], b[N][3], p[N][3];
#pragma unroll
    for (int j = 0; j < N; ++j) {
        const int l = Q::lev(j);
        load3(A.lv[l].T(), A.lv[l].pitch, gx[j], x[j]);
    }
#pragma unroll
    for (int j = 0; j < N; ++j)
        load3(Q::lev(j) == 1 ? A.rhsn2 : A.lv[Q::lev(j)].RHSN(), A.lv[Q::lev(j)].pitch, gx[j], b[j]);
#pragma unroll
    for (int j = 0; j < N; ++j)
        if (ok[j] && (A.keep & kKeepCoarse)) store3(A.lv[Q::lev(j)].RHS(), A.lv[Q::lev(j)].pitch, gx[j], b[j]);
    stamp<kMTc>(A, 1);
    // ---- phase A: restriction-leg smoother call of every level (:331), then get_residual (:338)
    for (int it = 0; it < ns; ++it) {
#pragma unroll
        for (int j = 0; j < N; ++j) {
            ST St;
            stc_of(j, St);
            copy3(p[j], x[j]);
            sweep(St, rdt, b[j], x[j]);
        }
    }
    stamp<kMTc>(A, 2);
#pragma unroll
    for (int j = 0; j < N; ++j) {
        const int l = Q::lev(j);
        const VLevel &V = A.lv[l];
        ST St;
        stc_of(j, St);
        double r[3];
        residual(St, rdt, p[j], b[j], r);
        if (ok[j] && (A.keep & kKeepCoarse)) store3(V.RES(), V.pitch, gx[j], r);
        if (l < C) {   // restriction-leg tnew: start of the prolongation leg and cascade target
            if (ok[j]) {
                const int i = t + 64 * Q::kk(j);
#pragma unroll
                for (int c = 0; c < 3; ++c) lds[Q::F(l) + c * Q::nt(l) + i] = p[j][c];
                lds[Q::M(l) + i] = div3(r[0] + r[1] + r[2]);
            }
        }
        copy3(x[j], p[j]);   // tnew_nonlin := tnew (:348 coarsest, :367 the others)
    }
    // restrictor of the next cycle (:336): RHSN_l(1, c) = mean(res(:, f3)),
    // (2, c) = mean(res(:, f4)), (3, c) = mean(res(:, f1)) (splitting.F90:10-32, 146-151)
    if constexpr (C >= 2) {
        __syncthreads();
#pragma unroll
        for (int j = 0; j < N; ++j) {
            const int l = Q::lev(j);
            if (l < 2 || !ok[j]) continue;
            const int i = t + 64 * Q::kk(j);   // children: 4i .. 4i+3 of level l - 1 (Level::pos)
            const double rn[3] = {lds[Q::M(l - 1) + 4 * i + 2], lds[Q::M(l - 1) + 4 * i + 3],
                                  lds[Q::M(l - 1) + 4 * i]};
            store3(A.lv[l].RHSN(), A.lv[l].pitch, gx[j], rn);
        }
    }
    stamp<kMTc>(A, 3);
    // ---- phase B: the n_coarse smoother calls of the coarsest level (:351-353) with the
    //      prolongation-leg call (:376) of every other level in its first n_smooth sweeps
    const int nB = ns * A.n_coarse;
    for (int it = 0; it < min(ns, nB); ++it) {
#pragma unroll
        for (int j = 0; j < N; ++j) {
            ST St;
            stc_of(j, St);
            copy3(p[j], x[j]);
            sweep(St, rdt, b[j], x[j]);
        }
    }
    for (int it = ns; it < nB; ++it) {   // the coarsest level alone
#pragma unroll
        for (int j = 0; j < N; ++j) {
            if (Q::lev(j) < C) continue;
            ST St;
            stc_of(j, St);
            copy3(p[j], x[j]);
            sweep(St, rdt, b[j], x[j]);
        }
    }
    stamp<kMTc>(A, 4);
#pragma unroll
    for (int j = 0; j < N; ++j) {
        const int l = Q::lev(j);
        const VLevel &V = A.lv[l];
        if (ok[j]) {
            store3(V.T(), V.pitch, gx[j], p[j]);
            if (l >= 2)
#pragma unroll
                for (int c = 0; c < 3; ++c) lds[Q::Y(l) + c * Q::nt(l) + t + 64 * Q::kk(j)] = p[j][c];
        }
    }
    // ---- prolongator (:370) among the coarse levels, on the LDS images of the
    //      restriction-leg tnew (its result is dead, :550)
    if constexpr (C >= 2) {
        __syncthreads();
#pragma unroll
        for (int j = 0; j < N; ++j) {
            const int l = Q::lev(j);   // coarse side l, fine side l - 1 >= 1
            if (l < 2 || !ok[j]) continue;
            const int i = t + 64 * Q::kk(j);
            const int fi[4] = {4 * i, 4 * i + 1, 4 * i + 2, 4 * i + 3};
            const double y[3] = {lds[Q::Y(l) + i], lds[Q::Y(l) + Q::nt(l) + i], lds[Q::Y(l) + 2 * Q::nt(l) + i]};
            prolong_cascade(lds + Q::F(l - 1), Q::nt(l - 1), fi, y);
        }
    }
    stamp<kMTc>(A, 7);
}

// ===================================================================== pipelined tail
// The coarse levels of the NEXT cycle, for the same tile, at the end of the level-1 launch
// (PIPE). The coarse-level work of cycle c+1 depends on cycle c only through level 2's RHS
// (the restrictor of cycle c's level-1 residual, :336) and on the coarse levels' own state,
// so the launch that finishes level 1 of cycle c can run the coarse levels of cycle c+1:
// level 2's RHS stays in the registers of the thread that restricts it and then smooths
// that sub-element, and level 2's tnew, read once, serves both the prolongator of cycle c
// (:370, its final value) and the start of cycle c+1 (:348). A call
// of n cycles is launched as coarse(1), [level 1 (c) + coarse (c+1)] for c < n, level 1 (n).
// Thread -> coarse element: level 2 on threads 0..nt(1)-1 (the owners of y1), the levels
// l >= 3 packed behind it (one wave for all of them at n_split = 5); the phases are the
// coarse launch's:
//   A: RHS_l := restrictor (:336), the restriction-leg call (:331), get_residual (:338);
//   B: restrictor of the new residuals into RHSN (next cycle), the prolongation-leg call
//      (:376) or, on the coarsest level, the 1 + n_coarse calls (:351-353), tnew stored;
//      then the prolongator cascade into the next finer level's image (:370; dead, :550).
template <int S, int L>
struct PGeo {
    using G = Geo<S, L>;
    static constexpr int C = G::C;
    static constexpr int nt(int l) { return G::nt(l); }
    static constexpr int T0(int l) { int o = 0; for (int i = 1; i < l; ++i) o += nt(i); return o; }
    static constexpr int NTH(int l) { return nt(l); }
    static_assert(T0(C + 1) <= G::MT, "coarse sub-elements exceed the threads of the tile");
    // LDS images in the F0 | M0 region: F_l, M_l (1 <= l < C)
    static constexpr int F(int l) { int o = 0; for (int i = 1; i < l; ++i) o += 3 * nt(i); return o; }
    static constexpr int M(int l) { int o = F(C); for (int i = 1; i < l; ++i) o += nt(i); return o; }
    static_assert(M(C) <= 4 * G::T, "coarse images exceed the level-1 image region");
    // the coarsest level's work runs at the start of the launch (coarsest_chain) when it does
    // not depend on the launch's level-1 residual (C >= 2); its final tnew waits for the
    // prolongator cascade in a stash behind the level-1 images. Measured (scripts/ab2.sh,
    // profiles/r01_v16_hoist_ab.txt): n_split = 5 full mesh 0.1324 -> 0.1300 ms per cycle,
    // N = 8 partition 0.0218 -> 0.0208, reference order 0.214 -> 0.202; n_split = 3 (16
    // un_eles per tile) 0.0127 -> 0.0131, so it stays off below n_split = 5
    static constexpr bool HOIST = C >= 2 && S >= 5;
    static constexpr int PC() { return 4 * G::T; }
    static constexpr int LDS() { return 4 * G::T + (HOIST ? 3 * nt(C) : 0); }
};

// The coarsest level of the next cycle, hoisted to the start of the pipelined launch (C >= 2):
// its restriction-leg call (:331 via :351), get_residual (:338) and the 1 + n_coarse calls
// (:351-353) read only its own tnew and its RHSN, both written by the previous launch -- its
// RHS is the restriction of level C-1's residual of the PREVIOUS cycle (:336) -- so the
// chain of 4 (1 + n_coarse) dependent sweeps runs on the coarsest level's threads while every
// thread's level-1 loads are in flight, instead of after the tile's level-1 work, as the
// launch's last phase. Phase B keeps what needs this launch: the restrictor into RHSN and
// the prolongator cascade. Loads first (coarsest_load), so that the level-1 loads issued
// behind them do not delay the chain.
template <int S, int L>
__device__ __forceinline__ bool coarsest_thread(int t) {
    using P = PGeo<S, L>;
    return t >= P::T0(L - 1) && t < P::T0(L - 1) + P::NTH(L - 1);
}
template <int S, int L>
__device__ __forceinline__ void coarsest_load(const VArgs &A, int t, int64_t tb, double x[3], double b[3]) {
    using G = Geo<S, L>;
    using P = PGeo<S, L>;
    constexpr int C = G::C;
    const VLevel &V = A.lv[C];
    const int i = t - P::T0(C);
    bool v;
    const uint32_t gx = tile_index<S>(A, tb, P::nt(C), C, i, v);
    load3(V.T(), V.pitch, gx, x);
    load3(V.RHSN(), V.pitch, gx, b);
}
template <int S, int L, class ST>
__device__ __forceinline__ void coarsest_chain(const VArgs &A, const double *__restrict__ sp, int t, int64_t tb,
                                               double x[3], const double b[3], double *lds) {
    using G = Geo<S, L>;
    using P = PGeo<S, L>;
    constexpr int C = G::C;
    const VLevel &V = A.lv[C];
    const double rdt = A.rdt;
    const int ns = A.n_smooth;
    const int i = t - P::T0(C);
    bool v;
    const uint32_t gx = tile_index<S>(A, tb, P::nt(C), C, i, v);
    const bool keep = A.keep & kKeepCoarse;
    if (v && keep) store3(V.RHS(), V.pitch, gx, b);
    ST St;
    stencil(G::uni(C), sp, gx >> G::lg(C), St);
    // the chain is the tile's critical path and the other waves are mostly waiting on HBM:
    // issue priority to it. Measured (scripts/ab2.sh, profiles/r01_v16_chain_prio.txt):
    // contracted arithmetic full mesh 0.1300 -> 0.1290 ms per cycle, N = 8 partition 0.0201 ->
    // 0.0195; the reference's order 0.1985 -> 0.2023 (its 3x fp64 work is not latency-bound
    // there), so only the contracted instance raises it
    constexpr int prio = std::is_same<ST, StcF>::value ? PAMG_CHAIN_PRIO : 0;
    if (prio) __builtin_amdgcn_s_setprio(prio);
    double p[3];
    sweeps1(St, rdt, ns, b, x, p);
    double r[3];
    residual(St, rdt, p, b, r);
    if (v && keep) store3(V.RES(), V.pitch, gx, r);
    copy3(x, p);   // tnew_nonlin := tnew (:348)
    const int nB = ns * A.n_coarse;
    sweeps1(St, rdt, nB, b, x, p);
    if (prio) __builtin_amdgcn_s_setprio(0);
    if (v) store3(V.T(), V.pitch, gx, p);
#pragma unroll
    for (int c = 0; c < 3; ++c) lds[P::PC() + c * P::nt(C) + i] = p[c];
}

template <int S, int L, class ST, bool HOIST>
__device__ __forceinline__ void coarse_next(const VArgs &A, const double *__restrict__ const *SP, int t, int64_t tb,
                                            const double y1[3], const double rn1[3], double *lds) {
    using G = Geo<S, L>;
    using P = PGeo<S, L>;
    constexpr int C = G::C;
    const double rdt = A.rdt;
    const int ns = A.n_smooth;
    double x[3], b[3], p[3];
    ST St;
    bool v = false;
    uint32_t gx = 0;
    int i = 0;
    __syncthreads();   // the level-1 images are dead
    // ---- phase A
    static_for<1, C + 1>([&](auto lc) {
        constexpr int l = decltype(lc)::value;
        if (t < P::T0(l) || t >= P::T0(l) + P::NTH(l)) return;   // wave-uniform
        const VLevel &V = A.lv[l];
        i = t - P::T0(l);
        gx = tile_index<S>(A, tb, P::nt(l), l, i, v);
        if constexpr (HOIST && l == C) return;   // phase A ran at the start of the launch (coarsest_chain)
        if constexpr (l == 1) {
            copy3(x, y1);   // final tnew of the previous cycle (:348 tnew_nonlin := tnew)
            copy3(b, rn1);  // the restriction of level 1's residual (:336)
        } else {
            load3(V.T(), V.pitch, gx, x);
            load3(V.RHSN(), V.pitch, gx, b);
        }
        const bool keep = A.keep & kKeepCoarse;
        if (v && keep) store3(V.RHS(), V.pitch, gx, b);
        stencil(G::uni(l), SP[l], gx >> G::lg(l), St);
        sweeps1(St, rdt, ns, b, x, p);
        double r[3];
        residual(St, rdt, p, b, r);
        if (v && keep) store3(V.RES(), V.pitch, gx, r);
        if constexpr (l < C) {
            if (v) {
#pragma unroll
                for (int c = 0; c < 3; ++c) lds[P::F(l) + c * P::nt(l) + i] = p[c];
                lds[P::M(l) + i] = div3(r[0] + r[1] + r[2]);
            }
        }
        copy3(x, p);   // tnew_nonlin := tnew (:348 coarsest, :367 the others)
    });
    __syncthreads();
    // ---- phase B
    static_for<1, C + 1>([&](auto lc) {
        constexpr int l = decltype(lc)::value;
        if (t < P::T0(l) || t >= P::T0(l) + P::NTH(l)) return;
        const VLevel &V = A.lv[l];
        // restrictor of the next cycle (splitting.F90:10-32, 146-151); the children of the tile's
        // sub-element i are 4i .. 4i+3 of level l - 1 (Level::pos)
        if constexpr (l >= 2) {
            if (v) {
                const double rn[3] = {lds[P::M(l - 1) + 4 * i + 2], lds[P::M(l - 1) + 4 * i + 3],
                                      lds[P::M(l - 1) + 4 * i]};
                store3(V.RHSN(), V.pitch, gx, rn);
            }
        }
        if constexpr (HOIST && l == C) {   // its 1 + n_coarse calls ran in coarsest_chain
#pragma unroll
            for (int c = 0; c < 3; ++c) p[c] = lds[P::PC() + c * P::nt(C) + i];
        } else {
            const int nB = l == C ? ns * A.n_coarse : ns;
            sweeps1(St, rdt, nB, b, x, p);
        }
        if (v) {
            if constexpr (!(HOIST && l == C)) store3(V.T(), V.pitch, gx, p);
            // ---- prolongator into level l - 1 (:370; result dead, :550) by the owner of the
            //      coarse sub-element, from its final tnew, on the restriction-leg image of
            //      level l - 1 (complete since the phase-A barrier; each child has one parent)
            if constexpr (l >= 2) {
                const int fi[4] = {4 * i, 4 * i + 1, 4 * i + 2, 4 * i + 3};
                prolong_cascade(lds + P::F(l - 1), P::nt(l - 1), fi, p);
            }
        }
    });
}

// ===================================================================== level 0
// Ownership: the adjacent pair 2t, 2t+1 of the tile (16-byte accesses, one un_ele,
// one operator record); for the prolongator, level-1 sub-element t.
template <int S, int L, class ST, bool PIPE, bool W8, bool RHSF = false>
__global__ __launch_bounds__(fine_mt(S), (S >= 3) ? ((W8 || fine_np(S) == 1) ? 8 : 4) : 2) void k_vc_fine(VArgs A, const double *__restrict__ sp0,
                                                                      const double *__restrict__ sp1,
                                                                      const double *__restrict__ sp2,
                                                                      const double *__restrict__ sp3,
                                                                      const double *__restrict__ sp4) {
    using G = Geo<S, L>;
    constexpr int C = G::C;
    static_assert(!PIPE || C > 0, "the pipelined launch needs a coarse level");
    // F0 | M0: restriction-leg tnew image and residual means (restrictor input) of level 1;
    // the pipelined tail reuses the region for the coarse levels' images
    constexpr int T = G::T, MT = G::MT, NP = G::NP;
    constexpr bool HOIST = PIPE && PGeo<S, L>::HOIST;
    __shared__ __attribute__((aligned(16))) double F0[C > 0 ? (PIPE ? PGeo<S, L>::LDS() : 4 * T) : 1];
    double *const M0 = F0 + 3 * T;
    const int t = threadIdx.x;
    const double rdt = A.rdt;
    const int ns = A.n_smooth;
    const int64_t tb = (int64_t)blockIdx.x + A.tile0;   // tile
    stamp<MT>(A, 0);
    stamp_hwid<MT>(A);
    const VLevel &V0 = A.lv[0];
    const bool keep1 = A.keep & kKeepL1, keeph = A.keep & kKeepHalo;
    bool v0;
    const uint32_t s0 = tile_index<S>(A, tb, T, 0, NP * t, v0);          // clamped: loads stay in bounds
    const uint32_t w0 = s0 >> G::lg(0);                                   // un_ele of the thread's sub-elements
    // ---- prologue
    int h0[NP];
#pragma unroll
    for (int k = 0; k < NP; ++k) h0[k] = v0 ? hs_pack(V0.H.hsub[(s0 + k) & ((1 << G::lg(0)) - 1)]) : 0;
    double x0[NP][3], b0[NP][3], p0[NP][3];
    double xc[3], bc[3];   // HOIST: the coarsest level's tnew and RHSN (coarsest_chain)
    if constexpr (HOIST)
        if (coarsest_thread<S, L>(t)) coarsest_load<S, L>(A, t, tb, xc, bc);
    if constexpr (RHSF) {
        // the start of a time step (:316-317, get_RHS :452-464): told := tnew and RHS from it
        // and the precomputed source term s', as k_rhs computes them (tnew_nonlin := tnew is
        // rewritten by :327 right here). kKeepTold: told stored and the step's constant halo
        // words written (k_overlap_static's); without it (a pamg_run step the next one
        // overwrites) both are dead
        static_assert(NP == 2, "RHSF launches stream pairs");
        double q0[3], q1[3];
        load3p<PAMG_NT_TL>(V0.T(), V0.pitch, s0, x0[0], x0[1]);
        load3p<PAMG_NT_RL>(V0.SRC(), V0.pitch, s0, q0, q1);
        const uint32_t wu = G::uni(0) ? (uint32_t)__builtin_amdgcn_readfirstlane(w0) : w0;
        const double c = sp0[(size_t)wu * kStcStride + kStcC];
        rhs_from_source(c, rdt, x0[0], q0, b0[0]);
        rhs_from_source(c, rdt, x0[1], q1, b0[1]);
        if (v0) {
            if (A.keep & kKeepTold) {
                store3p(V0.TOLD(), V0.pitch, s0, x0[0], x0[1]);
#pragma unroll
                for (int k = 0; k < NP; ++k) hs_write_static(V0.H, A.send_b, w0, h0[k], x0[k]);
            }
            store3p(V0.RHS(), V0.pitch, s0, b0[0], b0[1]);
        }
    } else if constexpr (NP == 2) {
        load3p<PAMG_NT_TL>(V0.T(), V0.pitch, s0, x0[0], x0[1]);      // tnew_nonlin := tnew (:327)
        load3p<PAMG_NT_RL>(V0.RHS(), V0.pitch, s0, b0[0], b0[1]);    // RHS of level 1 (get_RHS, constant in the time step)
    } else {
        load3(V0.T(), V0.pitch, s0, x0[0]);
        load3(V0.RHS(), V0.pitch, s0, b0[0]);
    }
    if constexpr (HOIST)
        if (coarsest_thread<S, L>(t)) coarsest_chain<S, L, ST>(A, G::C == 1 ? sp1 : G::C == 2 ? sp2 : G::C == 3 ? sp3 : sp4,
                                                               t, tb, xc, bc, F0);
    ST St;
    stencil(G::uni(0), sp0, w0, St);
    // ---- restriction leg: smoother (:331), get_residual (:338)
    if constexpr (NP == 2) sweeps2(St, rdt, ns, b0[0], b0[1], x0[0], x0[1], p0[0], p0[1]);
    else sweepsN<1>(St, rdt, ns, b0, x0, p0);
    stamp<MT>(A, 1);
    if (v0) {
        double r[NP][3];
#pragma unroll
        for (int k = 0; k < NP; ++k) residual(St, rdt, p0[k], b0[k], r[k]);
        if constexpr (NP == 2) {
            if constexpr (C > 0)
#pragma unroll
                for (int c = 0; c < 3; ++c)
                    *reinterpret_cast<double2 *>(F0 + c * T + 2 * t) = make_double2(p0[0][c], p0[1][c]);
            if (keep1) store3p(V0.RES(), V0.pitch, s0, r[0], r[1]);
            if constexpr (C > 0)   // restrictor input: mean of the residual components (splitting.F90:146-151)
                *reinterpret_cast<double2 *>(M0 + 2 * t) =
                    make_double2(div3(r[0][0] + r[0][1] + r[0][2]), div3(r[1][0] + r[1][1] + r[1][2]));
        } else {
            if constexpr (C > 0)
#pragma unroll
                for (int c = 0; c < 3; ++c) F0[c * T + t] = p0[0][c];
            if (keep1) store3(V0.RES(), V0.pitch, s0, r[0]);
            if constexpr (C > 0) M0[t] = div3(r[0][0] + r[0][1] + r[0][2]);
        }
    }
    stamp<MT>(A, 2);
    // level-1 sub-element j1 of the tile: its final tnew (coarse launch) for the prolongator,
    // fetched behind the prolongation-leg sweeps; its children are 4 j1 .. 4 j1 + 3 of the tile
    // (Level::pos) (threads 0..nt(1)-1: prolongator of sub-element t; the others: restrictor of
    //  t - nt(1); PIPE: both on threads 0..nt(1)-1)
    const int j1 = t & (G::nt(1) - 1);
    const bool casc = t < G::nt(1);
    bool v1 = false;
    uint32_t s1 = 0;
    double y1[3] = {0.0, 0.0, 0.0};
    if constexpr (C > 0) {
        s1 = tile_index<S>(A, tb, G::nt(1), 1, j1, v1);
        if (casc) load3(A.lv[1].T(), A.lv[1].pitch, s1, y1);
    }
    // ---- prolongation leg (:367-376) from the restriction-leg tnew; with one level,
    //      the 15 coarse smoother calls (:344-359)
#pragma unroll
    for (int k = 0; k < NP; ++k) copy3(x0[k], p0[k]);
    if constexpr (NP == 2) sweeps2(St, rdt, C > 0 ? ns : ns * A.n_coarse, b0[0], b0[1], x0[0], x0[1], p0[0], p0[1]);
    else sweepsN<1>(St, rdt, C > 0 ? ns : ns * A.n_coarse, b0, x0, p0);
    stamp<MT>(A, 3);
    if (v0) {
        // the cycle's halo words (update_overlaps, :555), all written here (see the header);
        // halo records by vector loads: the boundary lanes are few, and scalar copies of the
        // records would push the kernel past 80 SGPRs (7 instead of 8 waves per SIMD)
#pragma unroll
        for (int k = 0; k < NP; ++k)
            if (keeph) hs_write(false, V0.H, w0, h0[k], p0[k]);
        if constexpr (NP == 2) {
            store3p<PAMG_NT_TS>(V0.T(), V0.pitch, s0, p0[0], p0[1]);
            if (keep1) store3p(V0.TNN(), V0.pitch, s0, x0[0], x0[1]);
        } else {
            store3(V0.T(), V0.pitch, s0, p0[0]);
            if (keep1) store3(V0.TNN(), V0.pitch, s0, x0[0]);
        }
    }
    stamp<MT>(A, 4);
    // ---- prolongator (:370) on the LDS image (its result is dead, :550), and the restrictor
    //      of the next cycle (:336) from this cycle's residual (splitting.F90:10-32)
    //      (PIPE: both on the owner of level-2 sub-element t, which keeps the restriction as
    //      its RHS for the next cycle's coarse levels)
    double rn[3] = {0.0, 0.0, 0.0};
    if constexpr (C > 0) {
        __syncthreads();
        if (v1) {
            if (casc) {
                const int fi[4] = {4 * j1, 4 * j1 + 1, 4 * j1 + 2, 4 * j1 + 3};
                prolong_cascade(F0, T, fi, y1);
            }
            if (PIPE ? casc : (!casc && t < 2 * G::nt(1))) {
                rn[0] = M0[4 * j1 + 2];
                rn[1] = M0[4 * j1 + 3];
                rn[2] = M0[4 * j1];
                if constexpr (!PIPE) store3(A.rhsn2, A.lv[1].pitch, s1, rn);
            }
        }
    }
    if constexpr (PIPE) {
        const double *__restrict__ SP[kMaxFusedLevels] = {sp0, sp1, sp2, sp3, sp4};
        if (PAMG_TAIL_PRIO) __builtin_amdgcn_s_setprio(PAMG_TAIL_PRIO);
        coarse_next<S, L, ST, HOIST>(A, SP, t, tb, y1, rn, F0);
    }
    stamp<MT>(A, 7);
}

// ===================================================================== resident call
// A whole pamg_vcycle call of m cycles in one launch (fused = 3, the resident form): a
// workgroup carries its tile through every cycle of the call with all of the tile's state
// on-chip. It can, because nothing of a V-cycle crosses a tile (see the header) and the
// cycle's data dependences only run from cycle c-1 to cycle c:
//   * level l's restriction-leg call (:331) starts from its own tnew (:327 / :348) and reads
//     as RHS the restriction of level l-1's residual of the PREVIOUS cycle (:336);
//   * its prolongation-leg call starts from its own restriction-leg tnew (:367), the
//     prolongated values being overwritten at its first sweep (:550);
// so in cycle c every level runs its calls at once, from registers: level 1 on every thread
// (the adjacent pair, as k_vc_fine), level l >= 2 on the threads PGeo assigns it (one coarse
// sub-element each, as the pipelined tail), the coarsest level's 1 + n_coarse calls at raised
// priority. The only values that cross threads inside a cycle are the residual means the
// restrictor (:336) reads: level l writes its means of cycle c into one of two LDS buffers
// (by cycle parity), and at the start of cycle c+1 every coarse owner forms its RHS from the
// finer level's means -- one barrier per cycle (a buffer's next writer runs two cycles on,
// behind the barrier its readers passed). The prolongator (:370) is not computed: its output,
// tracer(l)%tnew, is overwritten by the smoother's first statement (tnew = tnew_nonlin, :550)
// before anything reads it (SURVEY.md A3 iv), and inside one launch no observer can run in
// between; the per-call API and the per-step kernels execute and store it.
// HBM sees the tile's state twice per call: loaded at the start (tnew and RHS or, starting
// a time step (RHSF), tnew and the source s' of level 1; tnew and RHSN of the coarse
// levels) and stored at the end, with the same final-cycle store policy as the pipelined
// launches (VArgs::keep). Every sweep, residual and restriction whose result is read runs,
// in the same order on the same values (a smoother call's last sweep, which only feeds a
// tnew_nonlin the cycle overwrites unread, is left to the compiler to drop): the state after
// the call is bitwise the per-step kernel sequence's (tests/test_gpu_parity.py). The cycle is
// fp64-issue-bound here, no longer HBM-bound.
#ifndef PAMG_RES_WAVES
#define PAMG_RES_WAVES 4
#endif
// n_split >= 5, L >= 3: the balanced-role instance k_vc_resb (A/B builds: 0 keeps k_vc_res)
#ifndef PAMG_RES_BALANCED
#define PAMG_RES_BALANCED 1
#endif
// (k_vc_resb keeps half of level 2 on wave 0: all of it on waves 6, 7 measured slower,
// profiles/r02_res_ab_variants.txt; two tiles per 1,024-thread workgroup measured equal,
// DESIGN.md 5)
template <int S, int L>
struct BGeo {
    using G = Geo<S, L>;
    static constexpr int C = G::C;
    // level l's residual means (0 <= l < C) in one parity buffer: level 1's T, then nt(1) ..
    static constexpr int MO(int l) { int o = 0; for (int i = 0; i < l; ++i) o += G::nt(i); return o; }
    static constexpr int MS = MO(C);
    static constexpr int LDS(bool rhsf) { return 2 * MS + (rhsf ? 3 * G::T : 0); }
};

// the operator records are re-fetched (scalar loads) where each phase uses them: an index the
// compiler cannot see through keeps it from hoisting every level's record out of the cycle
// loop into SGPRs it does not have (they spilled to VGPRs)
__device__ __forceinline__ uint32_t opaque(uint32_t u) {
    __asm__ volatile("" : "+v"(u));
    return u;
}

template <int S, int L, class ST, bool RHSF, bool XC = false>
__global__ __launch_bounds__(fine_mt(S), PAMG_RES_WAVES) void k_vc_res(VArgs A, const double *__restrict__ sp0,
                                                                      const double *__restrict__ sp1,
                                                                      const double *__restrict__ sp2,
                                                                      const double *__restrict__ sp3,
                                                                      const double *__restrict__ sp4) {
    using G = Geo<S, L>;
    using P = PGeo<S, L>;
    using B = BGeo<S, L>;
    constexpr int C = G::C;
    static_assert(C > 0 && G::NP == 2, "the resident launch needs a coarse level and streams pairs");
    constexpr int T = G::T, NP = 2;
    __shared__ __attribute__((aligned(16))) double MB[2 * B::MS];   // residual means, two parities
    auto means = [&](int c, int l) { return MB + (c & 1) * B::MS + B::MO(l); };
    const double *__restrict__ SP[kMaxFusedLevels] = {sp0, sp1, sp2, sp3, sp4};
    const int t = threadIdx.x;
    const double rdt = A.rdt;
    const int ns = A.n_smooth, m = A.cycles;
    const int64_t tb = resident_tile(A);   // tile
    const bool xe = !XC && A.xe_done != nullptr;   // the per-call exchange starts when the remote tiles end
    const bool xr = (XC || xe) && tile_remote<S, T>(A, tb);
    const VLevel &V0 = A.lv[0];
    const bool keep1 = A.keep & kKeepL1, keeph = A.keep & kKeepHalo, keepc = A.keep & kKeepCoarse;
    bool v0;
    const uint32_t s0 = tile_index<S>(A, tb, T, 0, NP * t, v0);   // clamped: loads stay in bounds
    const uint32_t w0 = s0 >> G::lg(0);
    int h0[NP];
#pragma unroll
    for (int k = 0; k < NP; ++k) h0[k] = v0 ? hs_pack(V0.H.hsub[(s0 + k) & ((1 << G::lg(0)) - 1)]) : 0;
    double x0[NP][3], b0[NP][3], p0[NP][3];
    double q[NP][3];   // RHSF: the source s' of the pair, every step's RHS reads it
    // Richardson (solver 2): get_residual rebuilds level 1's RHS from told (:865-867, get_RHS
    // :452-464) -- the smoother's first call of a time step still reads the RHS it had (its update
    // never calls get_RHS), every later use the rebuilt one: bn, switched in before the step's
    // first residual (pend)
    constexpr bool RICH = std::is_same<ST, StcR>::value;
    double bn[NP][3];
    bool pend = false;
    // the start of a time step (:316-317, get_RHS :452-464): told := tnew (t holds it) and the
    // RHS from it and s'; the run's last step stores told, the step's constant halo words
    // (kKeepTold) and the RHS it formed (kKeepL1) -- earlier steps' are overwritten unread
    auto start_step = [&](const double (&tn)[NP][3], bool last_step) {
        if constexpr (RHSF) {
            const uint32_t wu = G::uni(0) ? (uint32_t)__builtin_amdgcn_readfirstlane(w0) : w0;
            const double c = sp0[(size_t)wu * kStcStride + kStcC];
            if constexpr (RICH) {
#pragma unroll
                for (int k = 0; k < NP; ++k) rhs_from_source(c, rdt, tn[k], q[k], bn[k]);
                pend = true;
            } else {
#pragma unroll
                for (int k = 0; k < NP; ++k) rhs_from_source(c, rdt, tn[k], q[k], b0[k]);
            }
            if (last_step && v0) {
                if (A.keep & kKeepTold) {
                    store3p(V0.TOLD(), V0.pitch, s0, tn[0], tn[1]);
#pragma unroll
                    for (int k = 0; k < NP; ++k) hs_write_static(V0.H, A.send_b, w0, h0[k], tn[k]);
                }
                // the RHS lives in registers for the call; stored for an observer (dead inside pamg_run)
                // (Richardson: from the call's last cycle, once it is the rebuilt one)
                if (keep1 && !RICH) store3p(V0.RHS(), V0.pitch, s0, b0[0], b0[1]);
            }
        }
    };
    // ---- level 1: tnew (tnew_nonlin := tnew, :327) and the RHS
    if constexpr (RHSF) {   // the start of a time step (:316-317, get_RHS :452-464), as k_vc_fine
        load3p<PAMG_NT_TL>(V0.T(), V0.pitch, s0, x0[0], x0[1]);
        load3p<PAMG_NT_RL>(V0.SRC(), V0.pitch, s0, q[0], q[1]);
        // Richardson: the step's first smoother call reads the RHS the previous get_residual built
        if constexpr (RICH) load3p(V0.RHS(), V0.pitch, s0, b0[0], b0[1]);
        start_step(x0, A.steps == 1);
    } else {
        load3p<PAMG_NT_TL>(V0.T(), V0.pitch, s0, x0[0], x0[1]);
        load3p<PAMG_NT_RL>(V0.RHS(), V0.pitch, s0, b0[0], b0[1]);
        if constexpr (RICH) {   // the RHS the call's first residual rebuilds from told and s'
            double to[NP][3];
            load3p(V0.TOLD(), V0.pitch, s0, to[0], to[1]);
            load3p(V0.SRC(), V0.pitch, s0, q[0], q[1]);
            const uint32_t wu = G::uni(0) ? (uint32_t)__builtin_amdgcn_readfirstlane(w0) : w0;
            const double c = sp0[(size_t)wu * kStcStride + kStcC];
#pragma unroll
            for (int k = 0; k < NP; ++k) rhs_from_source(c, rdt, to[k], q[k], bn[k]);
            pend = true;
        }
    }
    // ---- the thread's coarse sub-element (level rl, tile-local ic): tnew and RHS of cycle 1
    //      (the RHS: RHSN, the restriction of the previous call's last residual)
    double xs[3] = {0.0, 0.0, 0.0}, bs[3] = {0.0, 0.0, 0.0};
    uint32_t gxc = 0;
    bool vc = false;
    int ic = 0;
    static_for<1, C + 1>([&](auto lc) {
        constexpr int l = decltype(lc)::value;
        if (t < P::T0(l) || t >= P::T0(l) + P::NTH(l)) return;
        const VLevel &V = A.lv[l];
        ic = t - P::T0(l);
        gxc = tile_index<S>(A, tb, P::nt(l), l, ic, vc);
        load3(V.T(), V.pitch, gxc, xs);
        load3(l == 1 ? A.rhsn2 : V.RHSN(), V.pitch, gxc, bs);
    });
    // the restrictor (:336): children 4 ic .. 4 ic + 3 on level l-1, cycle c (element_conversion order)
    auto restrict_rhs = [&](int c, int l, double b[3]) {
        const double *Mf = means(c, l - 1);
        b[0] = Mf[4 * ic + 2];
        b[1] = Mf[4 * ic + 3];
        b[2] = Mf[4 * ic];
    };
    // one cycle; LAST: the call's last, which makes the final-cycle stores (peeled, so that no
    // store address stays live across the loop)
    auto cycle = [&](int c, auto lastc) {
        constexpr bool last = decltype(lastc)::value;
        // ---- every coarse owner: its RHS of this cycle, the restriction of the finer level's
        //      residual of the previous cycle (the first cycle's is RHSN)
        if (c > 0)
            static_for<1, C + 1>([&](auto lc) {
                constexpr int l = decltype(lc)::value;
                if (t < P::T0(l) || t >= P::T0(l) + P::NTH(l) || !vc) return;
                restrict_rhs(c - 1, l, bs);
            });
        // ---- the coarsest level: restriction-leg call (:331 via :351), get_residual (:338),
        //      the 1 + n_coarse calls (:351-353) -- the tile's longest dependent chain, first
        if (t >= P::T0(C) && t < P::T0(C) + P::NTH(C)) {
            const VLevel &V = A.lv[C];
            ST St;
            stencil(G::uni(C), SP[C], opaque(gxc >> G::lg(C)), St);
            constexpr int prio = std::is_same<ST, StcF>::value ? PAMG_CHAIN_PRIO : 0;
            if (prio) __builtin_amdgcn_s_setprio(prio);
            if (last && keepc && vc) store3(V.RHS(), V.pitch, gxc, bs);
            double x[3], p[3];
            copy3(x, xs);
            sweeps1(St, rdt, ns, bs, x, p);
            double r[3];
            residual(St, rdt, p, bs, r);
            if (last && keepc && vc) store3(V.RES(), V.pitch, gxc, r);
            copy3(x, p);   // tnew_nonlin := tnew (:348)
            const int nB = ns * A.n_coarse;
            sweeps1(St, rdt, nB, bs, x, p);
            copy3(xs, p);
            if (prio) __builtin_amdgcn_s_setprio(0);
            if (last && vc) store3(V.T(), V.pitch, gxc, xs);
        }
        // ---- level 1: restriction-leg call (:331), get_residual (:338), prolongation-leg call
        //      (:367-376) from the restriction-leg tnew
        if (c > 0) {
#pragma unroll
            for (int k = 0; k < NP; ++k) copy3(x0[k], p0[k]);   // tnew_nonlin := tnew (:327)
        }
        ST St0;
        stencil(G::uni(0), sp0, opaque(w0), St0);
        sweeps2(St0, rdt, ns, b0[0], b0[1], x0[0], x0[1], p0[0], p0[1]);
        if constexpr (RICH)
            if (pend) {   // get_residual's get_RHS (:865-867): the rebuilt RHS from here on
#pragma unroll
                for (int k = 0; k < NP; ++k) copy3(b0[k], bn[k]);
                pend = false;
            }
        if (last && RICH && keep1 && v0) store3p(V0.RHS(), V0.pitch, s0, b0[0], b0[1]);
        if (v0) {
            double r[NP][3];
#pragma unroll
            for (int k = 0; k < NP; ++k) residual(St0, rdt, p0[k], b0[k], r[k]);
            if (last && keep1) store3p(V0.RES(), V0.pitch, s0, r[0], r[1]);
            *reinterpret_cast<double2 *>(means(c, 0) + 2 * t) =
                make_double2(div3(r[0][0] + r[0][1] + r[0][2]), div3(r[1][0] + r[1][1] + r[1][2]));
        }
#pragma unroll
        for (int k = 0; k < NP; ++k) copy3(x0[k], p0[k]);
        sweeps2(St0, rdt, ns, b0[0], b0[1], x0[0], x0[1], p0[0], p0[1]);
        if (last && v0) {
#pragma unroll
            for (int k = 0; k < NP; ++k)
                if (keeph) hs_write(false, V0.H, w0, h0[k], p0[k]);
            store3p<PAMG_NT_TS>(V0.T(), V0.pitch, s0, p0[0], p0[1]);
            if (keep1) store3p(V0.TNN(), V0.pitch, s0, x0[0], x0[1]);
        }
        if constexpr (XC && !last)   // the cycle's remote halo words, exchanged while the next cycles run
            if (xr && v0) {
#pragma unroll
                for (int k = 0; k < NP; ++k) hs_ring(G::uni(0), V0.H, A.ring + c * A.ring_stride, w0, h0[k], p0[k]);
            }
        // ---- levels 2 .. C-1 (1-based): both smoother calls and get_residual of the cycle
        static_for<1, C>([&](auto lc) {
            constexpr int l = decltype(lc)::value;
            if (t < P::T0(l) || t >= P::T0(l) + P::NTH(l)) return;   // wave-uniform
            const VLevel &V = A.lv[l];
            ST St;
            stencil(G::uni(l), SP[l], opaque(gxc >> G::lg(l)), St);
            if (last && keepc && vc) store3(V.RHS(), V.pitch, gxc, bs);
            double x[3], p[3];
            copy3(x, xs);
            sweeps1(St, rdt, ns, bs, x, p);
            double r[3];
            residual(St, rdt, p, bs, r);
            if (last && keepc && vc) store3(V.RES(), V.pitch, gxc, r);
            if (vc) means(c, l)[ic] = div3(r[0] + r[1] + r[2]);
            copy3(x, p);   // tnew_nonlin := tnew (:367)
            sweeps1(St, rdt, ns, bs, x, p);
            copy3(xs, p);
            if (last && vc) store3(V.T(), V.pitch, gxc, xs);
        });
        if constexpr (XC && !last)
            if (xr) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the ring words drained
        if constexpr (last)
            if (xe && xr) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the send words drained
        __syncthreads();
        if constexpr (XC && !last)
            if (t == 0) xc_signal(A, c);
        if constexpr (last)
            if (xe && xr && t == 0) xe_signal(A);
        // ---- after the call's last cycle: every coarse owner's RHSN, the restriction of the
        //      finer level's residual of that cycle (the next call's first RHS)
        if (last)
            static_for<1, C + 1>([&](auto lc) {
                constexpr int l = decltype(lc)::value;
                if (t < P::T0(l) || t >= P::T0(l) + P::NTH(l) || !vc) return;
                double bn[3];
                restrict_rhs(c, l, bn);
                store3(l == 1 ? A.rhsn2 : A.lv[l].RHSN(), A.lv[l].pitch, gxc, bn);
            });
    };
    // RHSF: A.steps time steps of m cycles; each later step starts from the tnew the previous
    // one left (p0: told := tnew, and tnew_nonlin := tnew at its first cycle, :316-317); the
    // run's last step start, which stores, is peeled out of the loop
    const int total = A.steps * m;
    int c = 0;
    if constexpr (RHSF) {
        for (int st = 0; st + 1 < A.steps; ++st) {
            if (st > 0) start_step(p0, false);
            for (int k = 0; k < m; ++k, ++c) cycle(c, std::false_type{});
        }
        if (A.steps > 1) start_step(p0, true);
    }
    for (; c + 1 < total; ++c) cycle(c, std::false_type{});
    cycle(total - 1, std::true_type{});
}

// ---- balanced roles (n_split >= 5, three levels or more). In k_vc_res the coarsest level's
// 1 + n_coarse calls (64 dependent sweeps at the defaults: a quarter of a tile's fp64 issue,
// on ONE wave -- an instruction stream does not get shorter with fewer active lanes) sit on
// wave 4 beside its level-1 pair, and wave 4 shares its SIMD with wave 0 (the hardware places
// waves w and w+4 of a 512-thread workgroup on one SIMD, scripts/micro/wave_simd.hip), which
// also carries level-2 work: that SIMD had ~2.3x the issue of the others and set the pace.
// Here a tile's issue is split evenly over its four SIMDs:
//   wave 4      the coarsest level alone;
//   wave 0      level 2: sub-elements 128..255, two per thread; the levels 3..L-1;
//   waves 1,2,3,5  level 1: an adjacent pair and a single sub-element per thread (768);
//   waves 6,7   level 1: an adjacent pair per thread (256), and level 2: sub-elements 0..127.
// Per tile-cycle (n_split 5, L 3), in units of 64 sub-elements x 2 smoother calls: SIMD(0,4)
// 64 sweeps on one wave (~5.4) + 2; SIMD(1,5) 6; SIMD(2,6), SIMD(3,7) 3 + 2 + 1. No thread holds
// two level-2 sub-elements beside its level-1 state (118 -> fewer VGPRs). A tile is one un_ele
// or a part of one (n_split >= 5), so every operator record is wave-uniform and every tile full.
//
// One barrier per cycle. The only values that cross threads inside a cycle are the residual
// means the restrictor (:336) reads: level l writes its means of cycle c, level l+1 reads them
// as the RHS of cycle c+1. They sit in two LDS buffers by cycle parity, so a level-(l+1) owner
// reads buffer (c-1) & 1 at the start of cycle c while level l fills buffer c & 1, and the
// barrier that closes cycle c is the only one needed (the next writer of a buffer, two cycles
// on, runs behind the barrier its readers passed). The prolongator (:370) is not computed here:
// its output, tracer(l)%tnew, is overwritten by the smoother's first statement
// (tnew = tnew_nonlin, :550) before anything reads it (SURVEY.md A3 iv), so within a resident
// call -- where no observer can run between :370 and :550 -- it is dead computation like a
// smoother call's last sweep; the per-call API and the per-step kernels execute
// and store it. Every operation whose result is read runs, in the same order on the same values:
// the state after the call is bitwise the per-step kernel sequence's (the same tests).
// three workgroups per CU (80 VGPRs; a few spilled words): 21,500 vs 20,330 V-cycles/s at two
// (scripts/ab_res.sh, profiles/r02_resm_ab.txt); L = 5 keeps two (it would spill 132 B per lane)
#ifndef PAMG_RESB_WAVES
#define PAMG_RESB_WAVES 6
#endif

template <int S, int L, class ST, bool RHSF, bool XC = false>
__global__ __launch_bounds__(512, L >= 5 ? PAMG_RES_WAVES : PAMG_RESB_WAVES) void k_vc_resb(VArgs A, const double *__restrict__ sp0,
                                                                const double *__restrict__ sp1,
                                                                const double *__restrict__ sp2,
                                                                const double *__restrict__ sp3,
                                                                const double *__restrict__ sp4) {
    using G = Geo<S, L>;
    using P = PGeo<S, L>;
    using B = BGeo<S, L>;
    constexpr int C = G::C, T = G::T;
    static_assert(C >= 2 && C <= 4 && T == 1024 && G::MT == 512 && S >= 5, "balanced roles: n_split >= 5, L 3..5");
    // two parity buffers of residual means; RHSF: the tile's source s' (3 T doubles) behind them
    // -- every step's RHS reads it; in registers it pushed the launch past 128 VGPRs
    __shared__ __attribute__((aligned(16))) double MB[B::LDS(RHSF)];
    double *const SQ = MB + 2 * B::MS;
    auto means = [&](int c, int l) { return MB + (c & 1) * B::MS + B::MO(l); };
    const int t = threadIdx.x;
    // the lane index, recomputed where it is used (mbcnt), so that it holds no VGPR across the loops
    auto lane_id = [] { return (int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); };
    const int wv = __builtin_amdgcn_readfirstlane(t >> 6);
    const double rdt = A.rdt;
    const int ns = A.n_smooth, m = A.cycles;
    // (Measured, not kept: starting the first round's k-th workgroup of a CU k x 1-2 us per cycle of the call late,
    // so that the co-resident tiles' loads and stores fall apart in time -- 0-4 % slower at 20 and 200 cycles,
    // profiles/r05_l_res_stagger.txt. A call's state crosses HBM once, ~250 us at one cycle, and is hidden under the
    // cycles from about five on: profiles/r05_k_call_fit.txt.)
    stamp<512>(A, 0);
    const int64_t tb = resident_tile(A);
    const bool xe = !XC && A.xe_done != nullptr;   // the per-call exchange starts when the remote tiles end
    const bool xr = (XC || xe) && tile_remote<S, T>(A, tb);
    const bool keep1 = A.keep & kKeepL1, keeph = A.keep & kKeepHalo, keepc = A.keep & kKeepCoarse;
    const int total = A.steps * m;
    // the restrictor (:336): the RHS of coarse sub-element i of level l from the means of its
    // children 4i .. 4i+3 (element_conversion's fin order) on level l-1, cycle c
    auto restrict_rhs = [&](int c, int l, int i, double b[3]) {
        const double *Mf = means(c, l - 1);
        b[0] = Mf[4 * i + 2];
        b[1] = Mf[4 * i + 3];
        b[2] = Mf[4 * i];
    };
    // Each role runs its own cycle loop with its own state (the loop is unswitched by role, so
    // the registers of one role's loop-carried state are not reserved in the others); every
    // role passes the same barrier once per cycle.
    //
    // level 2 (0-based 1), K = 1 or 2 adjacent sub-elements i0 .. i0+K-1 of the tile: load (tnew,
    // and the RHS: RHSN), the cycle's RHS (restrictor), both smoother calls + get_residual + means
    auto l2_load = [&](auto kc, int i0, double (&xs)[2][3], double (&bs)[2][3], uint32_t &gc, bool &vc) {
        constexpr int K = decltype(kc)::value;
        const VLevel &V = A.lv[1];
        gc = tile_index<S>(A, tb, P::nt(1), 1, i0, vc);
        if constexpr (K == 2) {
            load3p(V.T(), V.pitch, gc, xs[0], xs[1]);
            load3p(A.rhsn2, V.pitch, gc, bs[0], bs[1]);
        } else {
            load3(V.T(), V.pitch, gc, xs[0]);
            load3(A.rhsn2, V.pitch, gc, bs[0]);
        }
    };
    auto l2_legs = [&](auto kc, auto lastc, int c, int i0, double (&xs)[2][3], double (&bs)[2][3], uint32_t gc,
                       bool vc) {
        constexpr int K = decltype(kc)::value;
        constexpr bool last = decltype(lastc)::value;
        const VLevel &V = A.lv[1];
        if (c > 0) {
#pragma unroll
            for (int k = 0; k < K; ++k) restrict_rhs(c - 1, 1, i0 + k, bs[k]);
        }
        ST St;
        stencil(true, sp1, opaque(gc >> G::lg(1)), St);
        if (last && keepc && vc) {
            const uint32_t g = opaque(gc);
            if constexpr (K == 2) store3p(V.RHS(), V.pitch, g, bs[0], bs[1]);
            else store3(V.RHS(), V.pitch, g, bs[0]);
        }
        sweeps_tnew<K>(St, rdt, ns, bs, xs);   // restriction-leg call (:331): its tnew, in place
        double rr[2][3];
#pragma unroll
        for (int k = 0; k < K; ++k) residual(St, rdt, xs[k], bs[k], rr[k]);   // :338
        if (vc) {
            double *M = means(c, 1);
            if constexpr (K == 2) {
                if (last && keepc) store3p(V.RES(), V.pitch, opaque(gc), rr[0], rr[1]);
                *reinterpret_cast<double2 *>(M + i0) =
                    make_double2(div3(rr[0][0] + rr[0][1] + rr[0][2]), div3(rr[1][0] + rr[1][1] + rr[1][2]));
            } else {
                if (last && keepc) store3(V.RES(), V.pitch, opaque(gc), rr[0]);
                M[i0] = div3(rr[0][0] + rr[0][1] + rr[0][2]);
            }
        }
        sweeps_tnew<K>(St, rdt, ns, bs, xs);   // prolongation-leg call (:367-376), from that tnew
        if (last && vc) {
            const uint32_t g = opaque(gc);
            if constexpr (K == 2) store3p(V.T(), V.pitch, g, xs[0], xs[1]);
            else store3(V.T(), V.pitch, g, xs[0]);
        }
    };
    // after the call's last cycle: level 2's RHSN, the restriction of that cycle's level-1 means
    auto l2_rhsn = [&](auto kc, int c, int i0, uint32_t gc, bool vc) {
        constexpr int K = decltype(kc)::value;
        if (!vc) return;
        double bn[2][3];
#pragma unroll
        for (int k = 0; k < K; ++k) restrict_rhs(c, 1, i0 + k, bn[k]);
        const uint32_t g = opaque(gc);
        if constexpr (K == 2) store3p(A.rhsn2, A.lv[1].pitch, g, bn[0], bn[1]);
        else store3(A.rhsn2, A.lv[1].pitch, g, bn[0]);
    };
    if (wv == 4) {
        // ---- the coarsest level: its restriction-leg call, get_residual, 1 + n_coarse calls
        const VLevel &V = A.lv[C];
        bool vc;
        const uint32_t gc = tile_index<S>(A, tb, P::nt(C), C, lane_id(), vc);
        double xs[3], bs[3];
        load3(V.T(), V.pitch, gc, xs);
        load3(V.RHSN(), V.pitch, gc, bs);
        auto cycle = [&](int c, auto lastc) {
            constexpr bool last = decltype(lastc)::value;
            if (c > 0 && vc) restrict_rhs(c - 1, C, lane_id(), bs);   // (:336) of level C-1's residual of cycle c-1
            ST St;
            stencil(true, C == 2 ? sp2 : C == 3 ? sp3 : sp4, opaque(gc >> G::lg(C)), St);
            constexpr int prio = std::is_same<ST, StcF>::value ? PAMG_CHAIN_PRIO : 0;
            if (prio) __builtin_amdgcn_s_setprio(prio);
            if (last && keepc && vc) store3(V.RHS(), V.pitch, gc, bs);
            double(*x1)[3] = reinterpret_cast<double(*)[3]>(xs);
            const double(*b1)[3] = reinterpret_cast<const double(*)[3]>(bs);
            sweeps_tnew<1>(St, rdt, ns, b1, x1);   // restriction-leg call: its tnew, in place
            double r[3];
            residual(St, rdt, xs, bs, r);
            if (last && keepc && vc) store3(V.RES(), V.pitch, gc, r);
            // the 1 + n_coarse calls (:351-353): one chain of n_smooth n_coarse sweeps from that tnew
            // (tnew_nonlin := tnew, :348); its final tnew
            sweeps_tnew<1>(St, rdt, ns * A.n_coarse, b1, x1);
            if (prio) __builtin_amdgcn_s_setprio(0);
            if (last && vc) store3(V.T(), V.pitch, gc, xs);
            __syncthreads();
            if (last && vc) {   // RHSN: the restriction of level C-1's residual of the last cycle
                double bn[3];
                restrict_rhs(c, C, lane_id(), bn);
                store3(V.RHSN(), V.pitch, gc, bn);
            }
        };
        for (int c = 0; c + 1 < total; ++c) cycle(c, std::false_type{});
        cycle(total - 1, std::true_type{});
        stamp<512>(A, 7);   // the role's end (diagnostics build)
    } else if (wv == 0) {
        // ---- level 2: sub-elements 128 + 2 lane, +1; levels 3 .. L-1 (1-based), one sub-element
        //      of each per lane (none with L = 3)
        const int i2 = 128 + 2 * lane_id();
        double x2[2][3], b2[2][3];
        uint32_t g2 = 0;
        bool v2 = false;
        l2_load(std::integral_constant<int, 2>{}, i2, x2, b2, g2, v2);
        double xs[2][3] = {}, bs[2][3] = {};
        uint32_t gc[2] = {0, 0};
        bool vc[2] = {false, false};
        static_for<2, C>([&](auto lc) {
            constexpr int l = decltype(lc)::value;
            const VLevel &V = A.lv[l];
            gc[l - 2] = tile_index<S>(A, tb, P::nt(l), l, lane_id(), vc[l - 2]);
            load3(V.T(), V.pitch, gc[l - 2], xs[l - 2]);
            load3(V.RHSN(), V.pitch, gc[l - 2], bs[l - 2]);
        });
        const double *__restrict__ SP[kMaxFusedLevels] = {sp0, sp1, sp2, sp3, sp4};
        auto cycle = [&](int c, auto lastc) {
            constexpr bool last = decltype(lastc)::value;
            l2_legs(std::integral_constant<int, 2>{}, lastc, c, i2, x2, b2, g2, v2);
            static_for<2, C>([&](auto lc) {
                constexpr int l = decltype(lc)::value, k = l - 2;
                const VLevel &V = A.lv[l];
                if (c > 0 && vc[k]) restrict_rhs(c - 1, l, lane_id(), bs[k]);
                ST St;
                stencil(true, SP[l], opaque(gc[k] >> G::lg(l)), St);
                if (last && keepc && vc[k]) store3(V.RHS(), V.pitch, gc[k], bs[k]);
                double(*x1)[3] = reinterpret_cast<double(*)[3]>(xs[k]);
                const double(*b1)[3] = reinterpret_cast<const double(*)[3]>(bs[k]);
                sweeps_tnew<1>(St, rdt, ns, b1, x1);   // restriction-leg call: its tnew, in place
                double r[3];
                residual(St, rdt, xs[k], bs[k], r);
                if (last && keepc && vc[k]) store3(V.RES(), V.pitch, gc[k], r);
                if (vc[k]) means(c, l)[lane_id()] = div3(r[0] + r[1] + r[2]);
                sweeps_tnew<1>(St, rdt, ns, b1, x1);   // prolongation-leg call (:367-376), from that tnew
                if (last && vc[k]) store3(V.T(), V.pitch, gc[k], xs[k]);
            });
            __syncthreads();
            if constexpr (XC && !last)
                if (lane_id() == 0) xc_signal(A, c);
            if constexpr (last)   // behind the barrier the level-1 waves passed with their send words drained
                if (xe && xr && lane_id() == 0) xe_signal(A);
            if (last) {
                l2_rhsn(std::integral_constant<int, 2>{}, c, i2, g2, v2);
                static_for<2, C>([&](auto lc) {
                    constexpr int l = decltype(lc)::value, k = l - 2;
                    if (!vc[k]) return;
                    double bn[3];
                    restrict_rhs(c, l, lane_id(), bn);
                    store3(A.lv[l].RHSN(), A.lv[l].pitch, gc[k], bn);
                });
            }
        };
        for (int c = 0; c + 1 < total; ++c) cycle(c, std::false_type{});
        cycle(total - 1, std::true_type{});
        stamp<512>(A, 7);   // the role's end (diagnostics build)
    } else {
        // ---- level 1 (the reference's): waves 1,2,3,5 an adjacent pair + a single sub-element
        //      per thread (N = 3), waves 6,7 a pair (N = 2) and one sub-element of level 2
        const bool grpB = wv >= 6;
        const VLevel &V0 = A.lv[0];
        constexpr int hmask = (1 << G::lg(0)) - 1;
        auto level1 = [&](auto nc) {
            constexpr int N = decltype(nc)::value;   // level-1 sub-elements of the thread
            const int ga = (wv == 5 ? 3 : wv - 1) * 64 + lane_id(), gb = (wv - 6) * 64 + lane_id();
            const int jp = N == 3 ? 2 * ga : 768 + 2 * gb, js = 512 + ga;
            bool vp, vq = false;
            const uint32_t sp = tile_index<S>(A, tb, T, 0, jp, vp);
            const uint32_t sq = N == 3 ? tile_index<S>(A, tb, T, 0, js, vq) : 0u;
            const uint32_t w0 = sp >> G::lg(0);   // the tile's un_ele
            double X0[N][3], B0[N][3];   // tnew (told := tnew, tnew_nonlin := tnew at a cycle's start) and RHS
            // the start of a time step (:316-317, get_RHS :452-464): told := tnew (X0 holds it) and
            // the RHS from it and s'; the run's last step stores told, the step's constant halo
            // words (kKeepTold) and the RHS it formed (kKeepL1) -- earlier steps' are overwritten
            auto start_step = [&](bool last_step) {
                if constexpr (RHSF) {
                    const double c = sp0[(size_t)__builtin_amdgcn_readfirstlane(w0) * kStcStride + kStcC];
#pragma unroll
                    for (int k = 0; k < N; ++k) {   // the thread's own s' words (written by it, no barrier)
                        const int j = k < 2 ? jp + k : js;
                        const double q3[3] = {SQ[j], SQ[T + j], SQ[2 * T + j]};
                        rhs_from_source(c, rdt, X0[k], q3, B0[k]);
                    }
                    if (!last_step) return;
                    if (vp) {
                        if (A.keep & kKeepTold) {
                            store3p(V0.TOLD(), V0.pitch, sp, X0[0], X0[1]);
#pragma unroll
                            for (int k = 0; k < 2; ++k)
                                hs_write_static(V0.H, A.send_b, w0, hs_pack(V0.H.hsub[(sp + k) & hmask]), X0[k]);
                        }
                        if (keep1) store3p(V0.RHS(), V0.pitch, sp, B0[0], B0[1]);
                    }
                    if constexpr (N == 3)
                        if (vq) {
                            if (A.keep & kKeepTold) {
                                store3(V0.TOLD(), V0.pitch, sq, X0[2]);
                                hs_write_static(V0.H, A.send_b, w0, hs_pack(V0.H.hsub[sq & hmask]), X0[2]);
                            }
                            if (keep1) store3(V0.RHS(), V0.pitch, sq, B0[2]);
                        }
                }
            };
            if constexpr (RHSF) {
                double Q[N][3];
                load3p<PAMG_NT_TL>(V0.T(), V0.pitch, sp, X0[0], X0[1]);
                load3p<PAMG_NT_RL>(V0.SRC(), V0.pitch, sp, Q[0], Q[1]);
                if constexpr (N == 3) {
                    load3(V0.T(), V0.pitch, sq, X0[2]);
                    load3(V0.SRC(), V0.pitch, sq, Q[2]);
                }
#pragma unroll
                for (int q = 0; q < 3; ++q) {
                    *reinterpret_cast<double2 *>(SQ + q * T + jp) = make_double2(Q[0][q], Q[1][q]);
                    if constexpr (N == 3) SQ[q * T + js] = Q[2][q];
                }
                start_step(A.steps == 1);
            } else {
                load3p<PAMG_NT_TL>(V0.T(), V0.pitch, sp, X0[0], X0[1]);
                load3p<PAMG_NT_RL>(V0.RHS(), V0.pitch, sp, B0[0], B0[1]);
                if constexpr (N == 3) {
                    load3(V0.T(), V0.pitch, sq, X0[2]);
                    load3(V0.RHS(), V0.pitch, sq, B0[2]);
                }
            }
            // level 2 (0-based 1), group B: sub-element gb (wave 0 has 128 .. 255)
            double xs[2][3], bs[2][3];
            bool vc = false;
            uint32_t gc = 0;
            if constexpr (N == 2) l2_load(std::integral_constant<int, 1>{}, gb, xs, bs, gc, vc);
            auto cycle = [&](int c, auto lastc) {
                constexpr bool last = decltype(lastc)::value;
                ST St0;
                stencil(true, sp0, opaque(w0), St0);
                // restriction-leg call (:331) from tnew (tnew_nonlin := tnew, :327): its tnew, in place
                sweeps_tnew<N>(St0, rdt, ns, B0, X0);
                double r[N][3];
#pragma unroll
                for (int k = 0; k < N; ++k) residual(St0, rdt, X0[k], B0[k], r[k]);   // :338
                double *M0 = means(c, 0);
                if (vp) {
                    *reinterpret_cast<double2 *>(M0 + jp) =
                        make_double2(div3(r[0][0] + r[0][1] + r[0][2]), div3(r[1][0] + r[1][1] + r[1][2]));
                    if (last && keep1) store3p(V0.RES(), V0.pitch, sp, r[0], r[1]);
                }
                if constexpr (N == 3)
                    if (vq) {
                        M0[js] = div3(r[2][0] + r[2][1] + r[2][2]);
                        if (last && keep1) store3(V0.RES(), V0.pitch, sq, r[2]);
                    }
                sweeps_tnew<N>(St0, rdt, ns, B0, X0);   // prolongation-leg call (:367-376): the cycle's tnew
                if constexpr (last) {
                    // the call's last cycle: tnew_nonlin is observable, so its last sweep runs
                    double Y0[N][3];
#pragma unroll
                    for (int k = 0; k < N; ++k) {
                        copy3(Y0[k], X0[k]);
                        if (ns > 0) sweep(St0, rdt, B0[k], Y0[k]);
                    }
                    if (vp) {
#pragma unroll
                        for (int k = 0; k < 2; ++k)
                            if (keeph) hs_write(true, V0.H, w0, hs_pack(V0.H.hsub[(sp + k) & hmask]), X0[k]);
                        store3p<PAMG_NT_TS>(V0.T(), V0.pitch, sp, X0[0], X0[1]);
                        if (keep1) store3p(V0.TNN(), V0.pitch, sp, Y0[0], Y0[1]);
                    }
                    if constexpr (N == 3)
                        if (vq) {
                            if (keeph) hs_write(true, V0.H, w0, hs_pack(V0.H.hsub[sq & hmask]), X0[2]);
                            store3(V0.T(), V0.pitch, sq, X0[2]);
                            if (keep1) store3(V0.TNN(), V0.pitch, sq, Y0[2]);
                        }
                }
                if constexpr (XC && !last) {   // the cycle's remote halo words, exchanged while the next cycles run
                    double *rg = A.ring + c * A.ring_stride;
                    if (xr && vp)
#pragma unroll
                        for (int k = 0; k < 2; ++k) hs_ring(true, V0.H, rg, w0, hs_pack(V0.H.hsub[(sp + k) & hmask]), X0[k]);
                    if constexpr (N == 3)
                        if (xr && vq) hs_ring(true, V0.H, rg, w0, hs_pack(V0.H.hsub[sq & hmask]), X0[2]);
                }
                if constexpr (N == 2) l2_legs(std::integral_constant<int, 1>{}, lastc, c, gb, xs, bs, gc, vc);
                if constexpr (XC && !last)
                    if (xr) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the ring words drained
                if constexpr (last)
                    if (xe && xr) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the send words drained
                __syncthreads();
                if constexpr (N == 2 && last) l2_rhsn(std::integral_constant<int, 1>{}, c, gb, gc, vc);
            };
            // RHSF: A.steps time steps of m cycles; each later step starts from the tnew the
            // previous one left (told := tnew, tnew_nonlin := tnew, :316-317). The last step, whose
            // start stores told, the RHS and the constant halo words, is peeled (so that none of its
            // store addresses stays live across the loop).
            int c = 0;
            if constexpr (RHSF) {
                for (int st = 0; st + 1 < A.steps; ++st) {
                    if (st > 0) start_step(false);
                    for (int k = 0; k < m; ++k, ++c) cycle(c, std::false_type{});
                }
                if (A.steps > 1) start_step(true);
            }
            for (; c + 1 < total; ++c) cycle(c, std::false_type{});
            cycle(total - 1, std::true_type{});
            stamp<512>(A, 7);   // the role's end (diagnostics build)
        };
        if (grpB) level1(std::integral_constant<int, 2>{});
        else level1(std::integral_constant<int, 3>{});
    }
}

// ===================================================================== resident corrected call
// The corrected V-cycle (pamg_params.cycle = 1; pamg_api.cpp vcycle_corrected,
// oracle orc_vcycle_corrected): the reference's levels, smoother (transport_tri_semi.F90:491-507),
// residual (:725-873, with the b - A x sign), restrictor (splitting.F90:10-32, 146-151) and the P1
// interpolation its prolongator cascade encodes (splitting.F90:59-88), with the defects of the
// reference's cycle (SURVEY.md A3 iii/iv) fixed: the restrictor acts on the fresh residual, coarse
// levels start from zero, the interpolated coarse correction is added to the iterate the next smoother
// call starts from. Unlike the reference's cycle every step depends on the one before it -- level l's
// post-smoothing needs level l+1's result of the same cycle -- so a tile cannot run its levels at once.
// It can still keep the whole cycle on-chip: every operation stays inside a tile (an un_ele's
// sub-elements of every level), so one workgroup carries its tile through all the cycles
// of a pamg_vcycle call, the state in registers, and only the values that cross threads go through LDS:
//   step 0          level 0 (the reference's level 1): n_smooth sweeps from tnew, the fresh residual
//                   b - A x, its means (the restrictor's input) into LDS;
//   step l < C      level l: RHS := restrictor of level l-1's means, tnew := 0, n_smooth sweeps, the
//                   residual's means into LDS;
//   step C          the coarsest level: RHS, tnew := 0, n_coarse smoother calls; tnew into LDS;
//   step 2C - l     level l (C > l >= 1): tnew += P tnew_{l+1} (from LDS), n_smooth sweeps, tnew into LDS;
//   step 2C         level 0: tnew += P tnew_1, n_smooth sweeps; the call's last cycle stores the state,
//                   the halo words of the last smoother call and the fine residual after the cycle.
// One barrier closes each step but the last (2C per cycle); a step's LDS buffer is rewritten only one
// cycle later, behind the barriers its readers passed. Threads: level 0 on all 512 (an adjacent pair
// each), level 1 on waves 4-7 (one sub-element per thread, one wave per SIMD: waves w and w + 4 share
// one), level l >= 2 on wave l - 2 -- no thread holds two coarse levels, and each role runs its own
// cycle loop (unswitched, so one role's loop-carried registers are not reserved in another's).
// Every sweep, residual, mean and interpolation is the per-step kernels' device code on the same
// values in the same order (pamg_kernels.hip k_smooth, k_residual<.., NEG>, k_restrict_tile,
// k_interp_add): the state after the call is bitwise the per-step sequence's (tests/test_corrected.py).
// eight waves per SIMD (64 VGPRs, 9 spilled, four workgroups per CU): 16,536 vs 14,892 V-cycles/s at six
// (74 VGPRs, three per CU) -- the serialized steps of a tile leave more to hide (profiles/r04_e_corr_ab.txt)
#ifndef PAMG_CORR_WAVES
#define PAMG_CORR_WAVES 8
#endif
template <int S, int L>
struct KGeo {
    using G = Geo<S, L>;
    static constexpr int C = G::C;
    // LDS: the residual means of levels 0 .. C-1, then the iterates of levels 1 .. C (3 planes each)
    static constexpr int MO(int l) { int o = 0; for (int i = 0; i < l; ++i) o += G::nt(i); return o; }
    static constexpr int TO(int l) { int o = MO(C); for (int i = 1; i < l; ++i) o += 3 * G::nt(i); return o; }
    static constexpr int SIZE = TO(C + 1);
};

// negated residual (the corrected cycle's b - A x, k_residual<.., NEG>) and the restrictor's mean of it
template <class ST>
__device__ __forceinline__ double neg_resid_mean(const ST &St, double rdt, const double x[3], const double b[3],
                                                 double n[3]) {
    double r[3];
    resid(St, rdt, x, b, r);
#pragma unroll
    for (int c = 0; c < 3; ++c) n[c] = -r[c];
    return div3(n[0] + n[1] + n[2]);
}

// tnew += P y for child q (0..3, element_conversion's order) of the coarse sub-element whose tnew is y
// (k_interp_add, the P1 interpolation of the prolongator cascade, splitting.F90:59-88)
__device__ __forceinline__ void interp_add(double x[3], int q, const double y[3]) {
    const double m20 = 0.5 * y[2] + 0.5 * y[0], m12 = 0.5 * y[1] + 0.5 * y[2], m01 = 0.5 * y[0] + 0.5 * y[1];
    double a0, a1, a2;
    switch (q) {
        case 0: a0 = m20; a1 = m12; a2 = y[2]; break;
        case 1: a0 = m12; a1 = m20; a2 = m01; break;
        case 2: a0 = y[0]; a1 = m01; a2 = m20; break;
        default: a0 = m01; a1 = y[1]; a2 = m12; break;
    }
    x[0] = x[0] + a0;
    x[1] = x[1] + a1;
    x[2] = x[2] + a2;
}

template <int S, int L, class ST>
__global__ __launch_bounds__(512, PAMG_CORR_WAVES) void k_vc_corr(VArgs A, const double *__restrict__ sp0,
                                                                  const double *__restrict__ sp1,
                                                                  const double *__restrict__ sp2,
                                                                  const double *__restrict__ sp3,
                                                                  const double *__restrict__ sp4) {
    using G = Geo<S, L>;
    using K = KGeo<S, L>;
    constexpr int C = G::C, T = G::T;
    static_assert(C >= 1 && C <= 4 && T == 1024 && G::MT == 512 && G::NP == 2, "corrected resident call: 1024-element tiles, L 2..5");
    __shared__ __attribute__((aligned(16))) double LB[K::SIZE];
    const double *__restrict__ SP[kMaxFusedLevels] = {sp0, sp1, sp2, sp3, sp4};
    const int t = threadIdx.x;
    const int wv = __builtin_amdgcn_readfirstlane(t >> 6);
    auto lane_id = [] { return (int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); };
    const double rdt = A.rdt;
    const int ns = A.n_smooth, m = A.cycles;
    const int64_t tb = (int64_t)blockIdx.x + A.tile0;
    const bool keeph = A.keep & kKeepHalo;
    const VLevel &V0 = A.lv[0];
    constexpr int hmask = (1 << G::lg(0)) - 1;
    // level 0: the thread's adjacent pair (tile-local 2t, 2t + 1): tnew and the RHS, for the whole call
    bool v0;
    const uint32_t s0 = tile_index<S>(A, tb, T, 0, 2 * t, v0);
    const uint32_t w0 = s0 >> G::lg(0);
    double x0[2][3], b0[2][3];
    load3p<PAMG_NT_TL>(V0.T(), V0.pitch, s0, x0[0], x0[1]);
    load3p<PAMG_NT_RL>(V0.RHS(), V0.pitch, s0, b0[0], b0[1]);
    // the role: the coarse level lo the thread owns (0: none) -- level 1 on waves 4-7, level l >= 2 on wave l-2
    auto role = [&](auto loc) {
        constexpr int lo = decltype(loc)::value;
        bool vs = false;
        uint32_t gs = 0;
        int is = 0;
        if constexpr (lo > 0) {
            is = lo == 1 ? t - 256 : lane_id();
            gs = tile_index<S>(A, tb, G::nt(lo), lo, is, vs);
        }
        double xs[3], bs[3];
        auto cycle = [&](auto lastc) {
            constexpr bool last = decltype(lastc)::value;
            // ---- step 0: level 0's pre-smoothing call (:331) from tnew, its fresh residual, the means
            {
                ST St;
                stencil(G::uni(0), sp0, opaque(w0), St);
                for (int it = 0; it < ns; ++it) {
                    sweep(St, rdt, b0[0], x0[0]);
                    sweep(St, rdt, b0[1], x0[1]);
                }
                double n[3];
                const double a = neg_resid_mean(St, rdt, x0[0], b0[0], n);
                const double b = neg_resid_mean(St, rdt, x0[1], b0[1], n);
                if (v0) *reinterpret_cast<double2 *>(LB + K::MO(0) + 2 * t) = make_double2(a, b);
            }
            __syncthreads();
            // ---- steps 1 .. C-1: level l from zero, RHS the restriction of level l-1's residual
            static_for<1, C>([&](auto lc) {
                constexpr int l = decltype(lc)::value;
                if constexpr (lo == l) {
                    const double *Mf = LB + K::MO(l - 1);
                    bs[0] = Mf[4 * is + 2];
                    bs[1] = Mf[4 * is + 3];
                    bs[2] = Mf[4 * is];
                    xs[0] = xs[1] = xs[2] = 0.0;
                    ST St;
                    stencil(G::uni(l), SP[l], opaque(gs >> G::lg(l)), St);
                    for (int it = 0; it < ns; ++it) sweep(St, rdt, bs, xs);
                    double n[3];
                    const double mn = neg_resid_mean(St, rdt, xs, bs, n);
                    if (vs) {
                        LB[K::MO(l) + is] = mn;
                        if (last) {
                            const VLevel &V = A.lv[l];
                            store3(V.RHS(), V.pitch, gs, bs);
                            store3(V.RES(), V.pitch, gs, n);
                        }
                    }
                }
                __syncthreads();
            });
            // ---- step C: the coarsest level from zero, its n_coarse smoother calls (:351-353)
            if constexpr (lo == C) {
                const double *Mf = LB + K::MO(C - 1);
                bs[0] = Mf[4 * is + 2];
                bs[1] = Mf[4 * is + 3];
                bs[2] = Mf[4 * is];
                xs[0] = xs[1] = xs[2] = 0.0;
                ST St;
                stencil(G::uni(C), SP[C], opaque(gs >> G::lg(C)), St);
                constexpr int prio = std::is_same<ST, StcF>::value ? PAMG_CHAIN_PRIO : 0;
                if (prio) __builtin_amdgcn_s_setprio(prio);
                const int nB = ns * A.n_coarse;
                for (int it = 0; it < nB; ++it) sweep(St, rdt, bs, xs);
                if (prio) __builtin_amdgcn_s_setprio(0);
                if (vs) {
#pragma unroll
                    for (int c = 0; c < 3; ++c) LB[K::TO(C) + c * G::nt(C) + is] = xs[c];
                    if (last) {
                        const VLevel &V = A.lv[C];
                        store3(V.RHS(), V.pitch, gs, bs);
                        store3(V.T(), V.pitch, gs, xs);
                        store3(V.TNN(), V.pitch, gs, xs);
                    }
                }
            }
            __syncthreads();
            // ---- steps C+1 .. 2C-1: level l = C-1 .. 1, the interpolated correction, n_smooth sweeps
            static_for<1, C>([&](auto jc) {
                constexpr int l = C - decltype(jc)::value;
                if constexpr (lo == l) {
                    const double *Y = LB + K::TO(l + 1);
                    const int pc = is >> 2;
                    const double y[3] = {Y[pc], Y[G::nt(l + 1) + pc], Y[2 * G::nt(l + 1) + pc]};
                    interp_add(xs, is & 3, y);
                    ST St;
                    stencil(G::uni(l), SP[l], opaque(gs >> G::lg(l)), St);
                    for (int it = 0; it < ns; ++it) sweep(St, rdt, bs, xs);
                    if (vs) {
#pragma unroll
                        for (int c = 0; c < 3; ++c) LB[K::TO(l) + c * G::nt(l) + is] = xs[c];
                        if (last) {
                            const VLevel &V = A.lv[l];
                            store3(V.T(), V.pitch, gs, xs);
                            store3(V.TNN(), V.pitch, gs, xs);
                        }
                    }
                }
                __syncthreads();
            });
            // ---- step 2C: level 0, the interpolated correction of level 1, the post-smoothing call (:376)
            {
                const double *Y = LB + K::TO(1);
                const int pc = t >> 1;   // the pair's coarse parent; children 2t & 3, 2t & 3 + 1
                const double y[3] = {Y[pc], Y[G::nt(1) + pc], Y[2 * G::nt(1) + pc]};
                interp_add(x0[0], (2 * t) & 3, y);
                interp_add(x0[1], ((2 * t) & 3) + 1, y);
                ST St;
                stencil(G::uni(0), sp0, opaque(w0), St);
                if constexpr (!last) {
                    for (int it = 0; it < ns; ++it) {
                        sweep(St, rdt, b0[0], x0[0]);
                        sweep(St, rdt, b0[1], x0[1]);
                    }
                } else {
                    // the call's last cycle: the halo words of the last smoother call (:555 of its last
                    // sweep: the iterate before it), tnew = tnew_nonlin, and the fine residual after the cycle
                    for (int it = 1; it < ns; ++it) {
                        sweep(St, rdt, b0[0], x0[0]);
                        sweep(St, rdt, b0[1], x0[1]);
                    }
                    if (v0 && keeph)
#pragma unroll
                        for (int k = 0; k < 2; ++k) hs_write(G::uni(0), V0.H, w0, hs_pack(V0.H.hsub[(s0 + k) & hmask]), x0[k]);
                    sweep(St, rdt, b0[0], x0[0]);
                    sweep(St, rdt, b0[1], x0[1]);
                    double n[2][3];
                    (void)neg_resid_mean(St, rdt, x0[0], b0[0], n[0]);
                    (void)neg_resid_mean(St, rdt, x0[1], b0[1], n[1]);
                    if (v0) {
                        store3p<PAMG_NT_TS>(V0.T(), V0.pitch, s0, x0[0], x0[1]);
                        store3p(V0.TNN(), V0.pitch, s0, x0[0], x0[1]);
                        store3p(V0.RES(), V0.pitch, s0, n[0], n[1]);
                    }
                }
            }
        };
        for (int c = 0; c + 1 < m; ++c) cycle(std::false_type{});
        cycle(std::true_type{});
    };
    if (t >= 256) role(std::integral_constant<int, 1>{});
    else if (C >= 2 && wv == 0) role(std::integral_constant<int, (C >= 2 ? 2 : 0)>{});
    else if (C >= 3 && wv == 1) role(std::integral_constant<int, (C >= 3 ? 3 : 0)>{});
    else if (C >= 4 && wv == 2) role(std::integral_constant<int, (C >= 4 ? 4 : 0)>{});
    else role(std::integral_constant<int, 0>{});
}

// a resident launch (one kernel per pamg_vcycle call)
template <class K>
void launch_resident_kernel(K k, unsigned grid, unsigned block, hipStream_t s, const VArgs &A) {
    hipLaunchKernelGGL(k, dim3(grid), dim3(block), 0, s, A, A.lv[0].stc, A.lv[1].stc, A.lv[2].stc, A.lv[3].stc,
                       A.lv[4].stc);
}

// part: 0 level 1 (k_vc_fine), 1 coarse levels (k_vc_coarse), 2 level 1 + next cycle's coarse levels
template <int S, int L, class ST, bool W8>
hipError_t launch_sltw(hipStream_t s, const VArgs &A, unsigned grid, int part) {
    if constexpr (std::is_same<ST, StcR>::value) {   // Richardson: the resident call only (k_vc_res)
        if constexpr (L >= 2 && fine_np(S) == 2) {
            if (part == 6)
                launch_resident_kernel(k_vc_res<S, L, ST, false, true>, grid, Geo<S, L>::MT, s, A);
            else if (part == 5)
                launch_resident_kernel(k_vc_res<S, L, ST, true>, grid, Geo<S, L>::MT, s, A);
            else if (part == 4)
                launch_resident_kernel(k_vc_res<S, L, ST, false>, grid, Geo<S, L>::MT, s, A);
            else
                return hipErrorInvalidValue;
            return hipGetLastError();
        }
        return hipErrorInvalidValue;
    } else if (part == 1) {
        if constexpr (L >= 2)
            hipLaunchKernelGGL((k_vc_coarse<S, L, ST>), dim3(grid), dim3(kMTc), 0, s, A, A.lv[1].stc, A.lv[2].stc,
                               A.lv[3].stc, A.lv[4].stc);
        else
            return hipErrorInvalidValue;
    } else if (part == 2) {
        if constexpr (L >= 2)
            hipLaunchKernelGGL((k_vc_fine<S, L, ST, true, W8>), dim3(grid), dim3(Geo<S, L>::MT), 0, s, A, A.lv[0].stc,
                               A.lv[1].stc, A.lv[2].stc, A.lv[3].stc, A.lv[4].stc);
        else
            return hipErrorInvalidValue;
    } else if (part == 3) {   // part 2 starting a time step (RHSF)
        if constexpr (L >= 2 && fine_np(S) == 2)
            hipLaunchKernelGGL((k_vc_fine<S, L, ST, true, W8, true>), dim3(grid), dim3(Geo<S, L>::MT), 0, s, A,
                               A.lv[0].stc, A.lv[1].stc, A.lv[2].stc, A.lv[3].stc, A.lv[4].stc);
        else
            return hipErrorInvalidValue;
    } else if (part == 7) {   // the resident corrected call (k_vc_corr)
        if constexpr (L >= 2 && fine_np(S) == 2 && fine_tl(S) == 10)
            launch_resident_kernel(k_vc_corr<S, L, ST>, grid, 512, s, A);
        else
            return hipErrorInvalidValue;
    } else if (part >= 4 && part <= 6) {   // the resident call (5: starting a time step; 6: exchange every cycle)
        if constexpr (PAMG_RES_BALANCED && S >= 5 && L >= 3) {
            if (part == 6)
                launch_resident_kernel(k_vc_resb<S, L, ST, false, true>, grid, 512, s, A);
            else if (part == 5)
                launch_resident_kernel(k_vc_resb<S, L, ST, true>, grid, 512, s, A);
            else
                launch_resident_kernel(k_vc_resb<S, L, ST, false>, grid, 512, s, A);
        } else if constexpr (L >= 2 && fine_np(S) == 2) {
            if (part == 6)
                launch_resident_kernel(k_vc_res<S, L, ST, false, true>, grid, Geo<S, L>::MT, s, A);
            else if (part == 5)
                launch_resident_kernel(k_vc_res<S, L, ST, true>, grid, Geo<S, L>::MT, s, A);
            else
                launch_resident_kernel(k_vc_res<S, L, ST, false>, grid, Geo<S, L>::MT, s, A);
        } else {
            return hipErrorInvalidValue;
        }
    } else {
        hipLaunchKernelGGL((k_vc_fine<S, L, ST, false, W8>), dim3(grid), dim3(Geo<S, L>::MT), 0, s, A, A.lv[0].stc, nullptr,
                           nullptr, nullptr, nullptr);
    }
    return hipGetLastError();
}

inline bool no_scratch(const void *kernel) {
    hipFuncAttributes a{};
    return hipFuncGetAttributes(&a, kernel) == hipSuccess && a.localSizeBytes == 0;
}

// the 64-VGPR instance only where it saves a round: more workgroups than 3 per CU, at most 4
// (at n_split = 3 the launch fits one round either way and the bounded instance is 50 %
// slower)
template <int S, int L, class ST>
hipError_t launch_slt(hipStream_t s, const VArgs &A, unsigned grid, int part) {
    static const long n_cu = [] {
        int dev = 0, n = 0;
        if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
            n = 256;
        return (long)n;
    }();
    // (the reference's operation order, Stc, issues 3x the fp64 work and gains from the extra
    // wave at any size: 0.2678 -> 0.2560 ms per full-mesh cycle)
    // (the pipelined launch without its dead-until-final stores, kKeep*, moves 72 instead of
    // 120 B per level-1 sub-element and gains from it too: 0.1377 -> 0.1328 ms per full-mesh
    // cycle, scripts/ab_probe.py)
    const long w8_max = (std::is_same<ST, Stc>::value || part >= 2) ? (1l << 40) : 4 * n_cu;
    // (and only instances that fit 64 VGPRs without scratch: several L >= 4 and n_split = 3
    // instances spill there and stay at their natural register count)
    if (part >= 4 || std::is_same<ST, StcR>::value) return launch_sltw<S, L, ST, false>(s, A, grid, part);
    if constexpr (S >= 3 && !std::is_same<ST, StcR>::value) {
        static const bool fits[3] = {no_scratch((const void *)k_vc_fine<S, L, ST, false, true>),
                                     L >= 2 && no_scratch((const void *)k_vc_fine<S, L, ST, (L >= 2), true>),
                                     L >= 2 && no_scratch((const void *)k_vc_fine<S, L, ST, (L >= 2), true, true>)};
        if (part != 1 && fine_mt(S) == 512 && (long)grid > 3 * n_cu && (long)grid <= w8_max &&
            fits[part == 3 ? 2 : part == 2 ? 1 : 0])
            return launch_sltw<S, L, ST, true>(s, A, grid, part);
    }
    return launch_sltw<S, L, ST, false>(s, A, grid, part);
}

// operator arithmetic (pamg_params.arith): the reference's order, or the contracted form
template <int S, int L>
hipError_t launch_sl(hipStream_t s, const VArgs &A, unsigned grid, int part, int arith) {
    // 2: Richardson (Level::richardson), the resident call only
    return arith == 2   ? launch_slt<S, L, StcR>(s, A, grid, part)
           : arith == 1 ? launch_slt<S, L, StcF>(s, A, grid, part)
                        : launch_slt<S, L, Stc>(s, A, grid, part);
}

template <int S>
hipError_t launch_s(hipStream_t s, const VArgs &A, unsigned grid, int L, int part, int ar) {
    switch (L) {
        case 1: return launch_sl<S, 1>(s, A, grid, part, ar);
        case 2: if constexpr (S >= 2) return launch_sl<S, 2>(s, A, grid, part, ar); break;
        case 3: if constexpr (S >= 3) return launch_sl<S, 3>(s, A, grid, part, ar); break;
        case 4: if constexpr (S >= 4) return launch_sl<S, 4>(s, A, grid, part, ar); break;
        case 5: if constexpr (S >= 5) return launch_sl<S, 5>(s, A, grid, part, ar); break;
    }
    return hipErrorInvalidValue;
}


}  // namespace
}  // namespace pamg
