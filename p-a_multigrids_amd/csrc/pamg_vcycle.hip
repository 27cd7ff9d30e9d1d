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
// This unit: the launch dispatcher (launch_part) and the entry points of pamg_internal.h; the
// kernels live in pamg_vcycle_impl.h, instantiated once per n_split (pamg_vcycle_s.hip).
#include "pamg_vcycle_impl.h"

namespace pamg {
// pamg_vcycle_s.hip, one translation unit per n_split
#define PAMG_VC_DECL(S) hipError_t launch_vcycle_s##S(hipStream_t s, vc::VArgs A, unsigned grid, int L, int part, int ar);
PAMG_VC_DECL(1) PAMG_VC_DECL(2) PAMG_VC_DECL(3) PAMG_VC_DECL(4) PAMG_VC_DECL(5) PAMG_VC_DECL(6) PAMG_VC_DECL(7)
PAMG_VC_DECL(8)
#undef PAMG_VC_DECL

namespace {

hipError_t launch_part(hipStream_t s, const Level *lv, int L, int U, int n_split, int n_smooth, int n_coarse,
                       double rdt, double *tov, double *tovo, double *send1, double *rhsn2, int part, int keep,
                       int ua, int ub, double *send_b = nullptr, int cycles = 1, int steps = 1,
                       const VArgs *xc = nullptr) {
    const bool coarse = part == 1;
    if (part >= 2 && L < 2) return hipErrorInvalidValue;
    if (part >= 4 && cycles < 1) return hipErrorInvalidValue;
    // part 6: the per-cycle exchange's ring; part 4 may carry the early per-call exchange (tile order,
    // remote-tile counter, signal)
    if ((part == 6 && (!xc || cycles < 2 || !xc->ring || !xc->xc_done || !xc->xc_sig)) ||
        (xc && part != 6 && (part != 4 || !xc->tile_map || !xc->xe_done || !xc->xc_sig)))
        return hipErrorInvalidValue;
    if (steps != 1 && !(part == 5 && steps > 1 && vcycle_resident_run_supported(n_split, L))) return hipErrorInvalidValue;
    if (!vcycle_fusable(lv, L, n_split, 1, 0, n_smooth)) return hipErrorInvalidValue;
    VArgs A{};
    for (int l = 0; l < L; ++l) {
        const Level &V = lv[l + 1];
        if (V.nsub != (1 << (2 * (n_split - l)))) return hipErrorInvalidValue;
        if ((uint64_t)V.pitch * 3 >= (1ull << 29)) return hipErrorInvalidValue;   // 32-bit byte offsets
        VLevel &o = A.lv[l];
        if (V.TNN != V.T + 3 * V.pitch || V.RHS != V.T + 6 * V.pitch || V.RES != V.T + 9 * V.pitch ||
            V.TOLD != V.T + 12 * V.pitch || (l != 1 && V.RHSN != V.T + 15 * V.pitch) ||
            (l == 0 && (part == 3 || part == 5) && V.SRC != V.T + 18 * V.pitch))
            return hipErrorInvalidValue;
        if (l == 1 && rhsn2 != V.T + 15 * V.pitch && (!V.RHSN_alt || rhsn2 != V.RHSN_alt)) return hipErrorInvalidValue;
        o.base = V.T; o.stc = V.stc;
        o.pitch = V.pitch;
        const HaloPlan &P = V.halo;
        o.H = HaloArgs{P.d_hsub, P.d_hface, P.d_bcv, P.d_told_halo, tov, tovo, (l == 0 && send1) ? send1 : P.d_send,
                       1 << V.isplit};
    }
    A.U = U;
    A.n_smooth = n_smooth;
    A.n_coarse = n_coarse;
    A.rdt = rdt;
    A.rhsn2 = rhsn2;
    A.keep = keep;
    A.send_b = send_b;
    A.cycles = cycles;
    A.steps = steps;

    // tile: 2**TL level-1 sub-elements, TL = fine_tl (level-1 launch) or CGeo's (coarse launch)
    const int TL = coarse ? (2 * n_split > 8 ? std::min(2 * n_split, kFineTLMax) : 8) : fine_tl(n_split);
    // un_eles [ua, ub) (ub < 0: all); ua on a tile boundary, ub too unless it is U
    if (ub < 0 || ub > U) ub = U;
    const int64_t fa = (int64_t)ua << (2 * n_split), fb = (int64_t)ub << (2 * n_split), tm = (1ll << TL) - 1;
    if (ua < 0 || (fa & tm) || (ub != U && (fb & tm))) return hipErrorInvalidValue;
    A.tile0 = fa >> TL;
    const unsigned grid = fb > fa ? (unsigned)((fb - fa + tm) >> TL) : 0u;
    if (grid == 0) return hipSuccess;
    if (xc && part == 6) {
        A.ring = xc->ring;
        A.ring_stride = xc->ring_stride;
        A.xc_done = xc->xc_done;
        A.xc_sig = xc->xc_sig;
        A.xc_grid = grid;
    } else if (xc) {   // the early exchange: the map covers the grid's tiles (tile0 = 0)
        if (A.tile0 != 0) return hipErrorInvalidValue;
        A.tile_map = xc->tile_map;
        A.xe_done = xc->xe_done;
        A.xe_n = xc->xe_n;
        A.xc_sig = xc->xc_sig;
    }
    // diagnostics: PAMG_VCYCLE_STAMPS=<file> appends every launch's phase timeline
    static const char *stamp_path = PAMG_STAMPS ? getenv("PAMG_VCYCLE_STAMPS") : nullptr;
    const int waves = coarse ? kMTc / 64 : fine_mt(n_split) / 64;
    const size_t nst = (size_t)grid * waves * kStampSlots;
    if (stamp_path) {
        hipError_t e = hipMalloc(&A.stamps, nst * sizeof(long long));
        if (e != hipSuccess) return e;
        e = hipMemsetAsync(A.stamps, 0, nst * sizeof(long long), s);
        if (e != hipSuccess) return e;
    }
    hipError_t e = hipErrorInvalidValue;
    const int ar = lv[1].richardson ? 2 : lv[1].arith;
    switch (n_split) {
        case 1: e = launch_vcycle_s1(s, A, grid, L, part, ar); break;
        case 2: e = launch_vcycle_s2(s, A, grid, L, part, ar); break;
        case 3: e = launch_vcycle_s3(s, A, grid, L, part, ar); break;
        case 4: e = launch_vcycle_s4(s, A, grid, L, part, ar); break;
        case 5: e = launch_vcycle_s5(s, A, grid, L, part, ar); break;
        case 6: e = launch_vcycle_s6(s, A, grid, L, part, ar); break;
        case 7: e = launch_vcycle_s7(s, A, grid, L, part, ar); break;
        case 8: e = launch_vcycle_s8(s, A, grid, L, part, ar); break;
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

// halo_mode 1 (the reference's schedule: the halo rewritten at every sweep, :555) fuses too: the
// words of a smoother call's last sweep are the only observable ones either way (nothing reads
// t_overlap inside a cycle), so the fused forms write them once with the same values (bitwise,
// test_fused_vcycle_halo_mode1_bitwise)
bool vcycle_fusable(const Level *lv, int L, int n_split, int solver, int halo_mode, int n_smooth) {
    (void)lv;
    return (halo_mode == 0 || halo_mode == 1) && n_smooth > 0 && L >= 1 && L <= kMaxFusedLevels &&
           n_split <= kMaxFusedSplit && n_split >= L &&
           (solver != 2 || vcycle_resident_supported(n_split, L));   // Richardson: the resident call only
}

hipError_t launch_vcycle_coarse(hipStream_t s, const Level *lv, int L, int U, int n_split, int n_smooth,
                                int n_coarse, double rdt, double *tov, double *tovo, const double *rhsn2, int ua,
                                int ub, int keep) {
    if (L < 2) return hipSuccess;
    return launch_part(s, lv, L, U, n_split, n_smooth, n_coarse, rdt, tov, tovo, nullptr, const_cast<double *>(rhsn2),
                       1, keep, ua, ub);
}

hipError_t launch_vcycle_fine(hipStream_t s, const Level *lv, int L, int U, int n_split, int n_smooth,
                              int n_coarse, double rdt, double *tov, double *tovo, double *send1, double *rhsn2,
                              bool pipe, int keep, int ua, int ub, bool rhsf, double *send_b) {
    if (rhsf && !pipe) return hipErrorInvalidValue;
    return launch_part(s, lv, L, U, n_split, n_smooth, n_coarse, rdt, tov, tovo, send1, L > 1 ? rhsn2 : nullptr,
                       pipe ? (rhsf ? 3 : 2) : 0, keep, ua, ub, send_b);
}

hipError_t launch_vcycle_resident(hipStream_t s, const Level *lv, int L, int U, int n_split, int n_smooth,
                                  int n_coarse, double rdt, double *tov, double *tovo, double *send1, double *rhsn2,
                                  int keep, bool rhsf, double *send_b, int cycles, int steps, const EarlyXc *xe) {
    VArgs X{};
    if (xe) {
        if (rhsf || steps != 1) return hipErrorInvalidValue;
        X.tile_map = xe->tile_map;
        X.xe_done = xe->done;
        X.xe_n = xe->target;
        X.xc_sig = xe->sig;
    }
    return launch_part(s, lv, L, U, n_split, n_smooth, n_coarse, rdt, tov, tovo, send1, rhsn2, rhsf ? 5 : 4, keep, 0, -1,
                       send_b, cycles, steps, xe ? &X : nullptr);
}

// the level-1 tiles of the resident launch and whether each holds a face whose neighbour is on another
// rank (tile_remote's test on the host, from the level's face records)
void vcycle_remote_tiles(const Level &L1, int U, int n_split, std::vector<char> &remote) {
    const int TL = fine_tl(n_split);
    const int64_t n1 = (int64_t)U << (2 * n_split), nt = (n1 + (1ll << TL) - 1) >> TL;
    remote.assign((size_t)nt, 0);
    for (int64_t b = 0; b < nt; ++b) {
        int64_t u0 = (b << TL) >> (2 * n_split), u1 = (((b + 1) << TL) - 1) >> (2 * n_split);
        if (u1 >= U) u1 = U - 1;
        for (int64_t u = u0; u <= u1 && !remote[b]; ++u)
            for (int f = 0; f < 3; ++f)
                if ((L1.halo.hface[3 * u + f].x & 3) == 2) remote[b] = 1;
    }
}

hipError_t launch_vcycle_resident_xc(hipStream_t s, const Level *lv, int L, int U, int n_split, int n_smooth,
                                     int n_coarse, double rdt, double *tov, double *tovo, double *send1,
                                     double *rhsn2, int keep, int cycles, double *ring, int64_t ring_stride,
                                     unsigned *xc_done, unsigned long long *xc_sig) {
    VArgs X{};
    X.ring = ring;
    X.ring_stride = ring_stride;
    X.xc_done = xc_done;
    X.xc_sig = xc_sig;
    return launch_part(s, lv, L, U, n_split, n_smooth, n_coarse, rdt, tov, tovo, send1, rhsn2, 6, keep, 0, -1, nullptr,
                       cycles, 1, &X);
}

// the resident corrected call (k_vc_corr): `cycles` corrected V-cycles in one launch
hipError_t launch_vcycle_corrected(hipStream_t s, const Level *lv, int L, int U, int n_split, int n_smooth,
                                   int n_coarse, double rdt, double *tov, double *tovo, double *send1, double *rhsn2,
                                   int keep, int cycles) {
    if (!vcycle_corrected_supported(n_split, L)) return hipErrorInvalidValue;
    return launch_part(s, lv, L, U, n_split, n_smooth, n_coarse, rdt, tov, tovo, send1, rhsn2, 7, keep, 0, -1, nullptr,
                       cycles, 1);
}

bool vcycle_corrected_supported(int n_split, int L) {
    return L >= 2 && L <= kMaxFusedLevels && n_split >= L && n_split <= kMaxFusedSplit && fine_np(n_split) == 2 &&
           fine_tl(n_split) == 10;
}

// several time steps in one resident launch (k_vc_resb, or k_vc_res below n_split 5 and at L = 2)
bool vcycle_resident_run_supported(int n_split, int L) {
    return L >= 2 && L <= kMaxFusedLevels && n_split <= kMaxFusedSplit && fine_np(n_split) == 2;
}

// the resident form: two levels or more, adjacent pairs (fine_np == 2)
bool vcycle_resident_supported(int n_split, int L) { return L >= 2 && fine_np(n_split) == 2; }

// the RHSF instance streams adjacent pairs (fine_np == 2; A/B builds with PAMG_NP1_MAX_S may not)
bool vcycle_rhsf_supported(int n_split) { return fine_np(n_split) == 2; }

// un_eles per level-1 tile (1 when a tile is a part of one un_ele, n_split >= 6)
int vcycle_tile_un_eles(int n_split) { return fine_tl(n_split) > 2 * n_split ? 1 << (fine_tl(n_split) - 2 * n_split) : 1; }

}  // namespace pamg
