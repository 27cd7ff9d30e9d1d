// Internal structures of libpamg (not part of the C-ABI).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>
#include <vector>

#include "../../include/pamg.h"

namespace pamg {

constexpr int kMaxLevels = 12;
constexpr int kMaxFusedLevels = 5;
constexpr int kMaxFusedSplit = 8;   // fused V-cycle instances: n_split <= 8 (a tile is a part of an un_ele at >= 6)

// Per (un_ele, level) operator record, fp64, 32 doubles = 256 B (two 128-B lines):
// M (3x3 row-major) | Kd (3x3 row-major) | w = omega / D (3) | c = M_12 |
// A = (1/dt) M + Kd (3x3 row-major, the contracted operator of arith = 1) | omega (the Richardson
// update's relaxation, solve_Richardson :511-518).
// M and Kd are get_un_ele_mass_stiff_diffvol (ShapFun_unstruc.F90:304-335) reduced as
// transport_tri_semi.F90:592-607; D is get_diagonal (:481-486); M = c [[2,1,1],[1,2,1],[1,1,2]]
// exactly (checked in level_stencil), which the smoother kernels use (pamg_device.h apply_A).
constexpr int kStcM = 0, kStcK = 9, kStcW = 18, kStcC = 21, kStcA = 22, kStcOm = 31, kStcStride = 32;

// Level-1 geometry record per un_ele (get_splitting, Msh2Tri.F90:69-107):
// x3, y3, v1x, v1y, v2x, v2y (v = edge / 2**i_split), pad to 8 doubles.
constexpr int kGeoStride = 8;

struct HaloCopy {     // update_overlaps copy entry (splitting.F90:1256-1391)
    int32_t src;      // global sub-element index (local numbering) on this rank
    int32_t dst;      // element offset in t_overlap (local) or in the send buffer
};
struct HaloBC {       // boundary entry (splitting.F90:1243-1252, :1287-1295, :1345-1353)
    int32_t dst_a, dst_b;
    double val_a, val_b;
};

struct HaloPlan {
    std::vector<HaloCopy> local;          // destination on this rank
    std::vector<HaloBC> bc;
    std::vector<HaloCopy> remote;         // dst = entry index in the packed send buffer
    std::vector<int> send_peer_off;       // per peer: first entry in `remote` (size npeers+1)
    std::vector<int> recv_dst;            // per received entry: t_overlap offset
    std::vector<int> recv_peer_off;       // per peer: first entry in recv (size npeers+1)
    std::vector<int> peers;               // peer ranks
    // fused form used by the smoother kernel (one record per owned un_ele and face, one
    // entry per sub-element of the level): the smoother threads that hold a boundary
    // sub-element write its halo words themselves.
    std::vector<int4> hface;              // (U*3) {mode | rev << 2, dst base, aux, 0}; mode 0 BC, 1 local, 2 remote
    std::vector<int4> hsub;               // (nsub) position i (1-based, 0 = none) along faces 1, 2, 3
    std::vector<double2> bcv;             // BC values sin(x+y) at the two face nodes, (u, f, i) order
    std::vector<int> surf;                // surf_ele(i, f) of loc_surf_ele_multigrid, (m, 3), 1-based
    int n_told = 0;                       // entries of the told halo (3 fp64 each); hface.w = first entry
    int4 *d_hface = nullptr, *d_hsub = nullptr;
    // the positions of the sub-elements that have halo words (any hsub face nonzero), ascending: the
    // words-only refresh (launch_face_words) runs over U x nbpos of them instead of the whole level
    int *d_bpos = nullptr;
    int nbpos = 0;
    double2 *d_bcv = nullptr;
    int *d_surf = nullptr;
    double *d_told_halo = nullptr;        // told values of the copied sub-elements, refreshed when told changes
    // device copies
    HaloCopy *d_local = nullptr, *d_remote = nullptr;
    HaloBC *d_bc = nullptr;
    int *d_recv_dst = nullptr;
    double *d_send = nullptr, *d_recv = nullptr;   // 6 doubles per entry (tnew 3, told 3)
    // second send buffer: the fused V-cycle packs cycle k+1 while cycle k's exchange is in
    // flight; send_cur = the buffer holding the last packed words
    double *d_send_b = nullptr;
    int send_cur = 0;
    // halo_exchange = 1 with the resident call: the tnew words of every cycle but the last, 3 per
    // remote entry, ring_cap cycles (on first use), and the receive side of one of them
    double *d_ring = nullptr, *d_recv3 = nullptr;
    int ring_cap = 0;
    double *send_buf(int i) const { return i ? d_send_b : d_send; }
};

struct Level {
    int isplit = 0;       // n_split - l + 1
    int nsub = 0;         // 4**isplit
    int64_t N = 0;        // nsub * U_local
    int64_t pitch = 0;    // plane stride (>= N, multiple of 64)
    // SoA planes [3][pitch]
    double *T = nullptr, *TNN = nullptr, *RHS = nullptr, *RES = nullptr, *TOLD = nullptr;
    // restrictor(l - 1) of the finer level's current residual, computed where that residual
    // is produced (fused V-cycle) and consumed as RHS by the next cycle (l >= 2)
    double *RHSN = nullptr;
    // level 2 only: the second RHSN buffer of the concurrent fused cycle (fused = 2), whose
    // level-1 launch writes the one the concurrent coarse launch is not reading
    double *RHSN_alt = nullptr;
    // level 1 only: the cascaded source term s' of get_RHS (:452-464, :593), M s with
    // s_j = -2k sin(x_j + y_j) at the sub-element nodes -- geometry only, formed once at upload
    // (k_source) and added to rdt M told by every RHS evaluation
    double *SRC = nullptr;
    double *stc = nullptr;            // U_local * kStcStride
    int2 *subinfo = nullptr;          // nsub: (irow, ipos) of get_str_info, by storage position
    // Storage order of the sub-elements of an un_ele: hierarchical, not the
    // reference's row-wise numbering -- the four children of the coarser level's sub-element at
    // position p (element_conversion, splitting.F90:97-140, in its order) sit at positions
    // 4p .. 4p+3, so over a whole level the children of global coarse index g are the global
    // fine indices 4g .. 4g+3, and every aligned block of 4**k sub-elements carries its own
    // coarser sub-elements. The coarsest level keeps the reference's order.
    // pos[e - 1] = storage position of the reference's str_ele e (host); d_pos on the device
    // for the (3, nsub, U) boundary layout converters.
    std::vector<int> pos;
    int *d_pos = nullptr;
    // face-coupled operator (pamg_params.op = 1): per storage position fnb = {the
    // neighbour's position across faces 1..3, or -sp (position along the un_ele face), up flag};
    // per local un_ele fface = {w_in[3], w_b[3], D0[3], pad} (kFaceStride doubles) and fsx[4] =
    // per un_ele face: S(F1) | S(F2) << 2 | domain boundary << 4
    int4 *fnb = nullptr;
    double *fface = nullptr;
    int *fsx = nullptr;
    // the colour lists of the red-black passes: the storage positions of the up sub-elements
    // (fnb.w != 0, ascending), then of the down ones -- nup + ndn = nsub
    int *cpos = nullptr;
    int4 *cnb = nullptr;   // fnb of the colour lists' positions (cnb[i] = fnb[cpos[i]]): one load, not two in a row
    int nup = 0, ndn = 0;
    // the two-sweep passes (k_face_pp): per (local un_ele, face, halo slot) the gather entry of the
    // neighbour's boundary sub-element e facing the slot -- {e's global index (-1 boundary face, -2 another
    // rank), then per face of e the global index of the value across it, -1 - p for this un_ele's own
    // position p, or -(1 + nsub + 3 bcv index + face - 1) for a boundary word}
    int4 *gtab = nullptr;
    // per gather entry the face pattern of e (bit fi: e's face fi is inner, fnb's sign): k_face_pp reads it beside the
    // entry instead of fnb[e] after it
    int *gpat = nullptr;
    // every sub-element with halo words (HaloPlan::hsub) is an up one: the chain publishes a
    // sweep's words right after its up pass (k_face_chain, early)
    bool words_up = false;
    int nui = 0;   // up sub-elements without halo words per un_ele: cpos lists them first among the ups
    double *Ainv = nullptr;           // U_local * 9: FINDInv of (1/dt) M + Kd (coarse_solver = 1)
    double *blocks = nullptr;         // assembled per-sub-element operator (lazy, pamg_sweep_bench)
    // the persistent face chain (pamg_face.hip k_face_chain; lazy): its workgroups' neighbour lists
    // (CSR over chain_g workgroups) and the flag words it polls (zeroed before every launch)
    int chain_g = 0;
    int *chain_nb_off = nullptr, *chain_nb_list = nullptr;
    unsigned *chain_flags = nullptr;
    size_t chain_flag_bytes = 0;
    // the flags' epoch: a chain call publishes epoch + s + 1 for its sweep s and the next call starts
    // past every value published, so the flags are zeroed only at setup and on wrap
    unsigned chain_epoch = 0;
    int arith = 0;                    // operator arithmetic of this level's kernels (pamg_params.arith)
    bool richardson = false;          // solver 2: the Richardson update (solve_Richardson, :511-518)
    HaloPlan halo;
};

struct Timing {
    unsigned mask = 0;
    // events around one launch in `stride` of each kernel class (the first, then every
    // stride-th): a HIP event pair costs ~10 us between back-to-back launches
    int stride = 1;
    long seq[PAMG_K_COUNT] = {0};
    struct Rec { int kid; hipEvent_t a, b; double bytes; };
    std::vector<Rec> pending;
    std::vector<hipEvent_t> pool;
    double ms[PAMG_K_COUNT] = {0};
    long count[PAMG_K_COUNT] = {0};
    double bytes[PAMG_K_COUNT] = {0};
};

struct Comm;  // pamg_comm.cpp

}  // namespace pamg

struct pamg_handle {
    pamg_params p{};
    int device = 0;
    hipStream_t stream = nullptr;
    int U = 0;                 // local un_ele count
    int U_global = 0;
    std::vector<int> owned;    // global ids (0-based) of local un_eles, ascending
    std::vector<double> Xo;    // X(2,3) of the local un_eles (pamg_write_vtu)
    pamg::Level lv[pamg::kMaxLevels + 1];   // 1-based
    double *geo1 = nullptr;    // U * kGeoStride
    double *tov = nullptr, *tovo = nullptr; // (slots, 3, U) t_overlap / t_overlap_old
    double *tov_b = nullptr;   // the second t_overlap buffer of the fused face-operator sweeps (on first use)
    int slots = 0;
    int tnn_level = 1;
    // t_overlap_old and the boundary words hold what level 1's smoother writes in this
    // time step (the fused V-cycle then writes only the tnew words); cleared by every
    // operation that writes or changes them otherwise
    bool overlap_static_l1 = false;
    // level 1's compact told copy of the halo is behind TOLD (pamg_run started a step without
    // refreshing it); the fused V-cycle's k_overlap_static writes it from TOLD
    bool told_halo_stale_l1 = false;
    // pamg_run: the coarse levels already ran the next call's first cycle (its last launch was
    // pipelined); that call skips its first coarse launch
    bool coarse_ahead = false;
    // pamg_run: this step's told := tnew and level-1 RHS are left to the first level-1 launch
    // of its fused V-cycle (RHSF)
    bool rhs_pending = false;
    // the fused V-cycle's halo exchange (RCCL) runs on stream_comm, overlapped with the next
    // cycle; joined back into `stream` before pamg_vcycle returns
    hipStream_t stream_comm = nullptr;
    hipEvent_t ev_packed = nullptr, ev_sent[2] = {nullptr, nullptr};
    bool sent_pending[2] = {false, false};
    // fused = 2: the coarse-level launch of each cycle runs on stream_c beside the level-1
    // launch on `stream`; ev_fine / ev_coarse order them across cycles (RHSN of level 2)
    hipStream_t stream_c = nullptr;
    int call_schedule = 0;   // pamg_set_call_schedule (0: automatic)
    hipEvent_t ev_fine = nullptr, ev_coarse = nullptr;
    // RHSN of every level holds the restriction of the finer level's current residual
    bool rhsn_valid = true;
    // op = 1, cycle 0, inside vcycle_face_pp (PAMG_FACE_RR): a streaming level l >= 2 folds its restrictor into the pass
    // that computes its residual (into level l+1's RHSN_alt, swapped in at the next cycle's restriction point);
    // pp_folded[l]: level l+1's RHSN_alt holds the restriction of level l's latest residual (face_restrict_prev)
    bool pp_fold = false;
    bool pp_folded[pamg::kMaxLevels + 1] = {};
    bool mesh_ready = false;
    std::string err;
    pamg::Timing timing;
    // multi-GPU
    int nranks = 1, rank = 0;
    std::vector<int> owner;    // global owner map (empty = all local)
    // self-peer plan (pamg_comm_init_self, one rank): virtual part of every un_ele; the halo
    // words across two parts go through the RCCL communicator to this rank itself
    std::vector<int> vpart;
    pamg::Comm *comm = nullptr;
    double *scratch = nullptr; size_t scratch_bytes = 0;
    // op = 1: the local un_eles' neighbours (0-based local ids, -1: none or another rank), 3 per un_ele
    std::vector<int> neig_local;
    unsigned *chain_tmo = nullptr;   // give-up word of the face chain's / wavefront's bounded spins
                                     // ([1..2] the chain's co-residency guard, [3] its aborts)
    bool chain_pending = false;      // a chain or wavefront launch ran since face_chain_check last read it
    // the guarded chain launches' gates (face_call, PAMG_CHAIN_GATE): the stream waits on `gate` (signal
    // memory) after each launch for the count the launch adds when it ran; an aborted one leaves the stream
    // waiting until the host has run the call's fallback (face_gates_drain) -- the host no longer waits for
    // each launch. gate_stat: pinned ring of the launches' reports (seq << 1 | aborted, kGateRing entries)
    unsigned long long *gate = nullptr, *gate_stat = nullptr;
    unsigned long long gate_seq = 1, gate_base = 0;   // next launch's tag; the gate's count so far
    struct GatePending {
        unsigned long long seq, want;
        int l, sweeps, run;
        bool dead_last, src_is_T, both;
        double *T, *TNN, *RHS;   // the level's buffers at the launch (level 2's RHS is swapped within a call)
    };
    std::vector<GatePending> gates;   // in stream order, not yet read back
    hipStream_t stream_fb = nullptr;  // the gated fallback's launches (the handle's stream waits at the gate)
    // the face operator's wavefront calls (k_face_wave; lazy, single domain): the ticket order (a
    // reverse Cuthill-McKee numbering of neig_local), its band, the neighbours on the device and the
    // per-un_ele flags + ticket counter
    int *wave_order = nullptr, *wave_neig = nullptr;
    unsigned *wave_flags = nullptr;
    int wave_band = -1;
    unsigned long long *wave_gran = nullptr;   // two granule buffers, 2 words per t_overlap double each
    unsigned wave_tag = 1;                     // tag base of the next wavefront launch
    // the resident call's per-cycle exchange (halo_exchange = 1): per-cycle workgroup counters and
    // the signal the comm stream waits on (cycles published so far: xc_sig_base after the last call)
    unsigned *xc_done = nullptr;
    int xc_cap = 0;
    unsigned long long *xc_sig = nullptr;
    unsigned long long xc_sig_base = 0;
    // the early per-call exchange of the resident call (halo_exchange = 0 on a partition): the tile
    // order with the remote tiles first (device, built on first use), their count, its counter
    int *xe_map = nullptr;
    int xe_nremote = -1;             // -1: not built
    unsigned *xe_done = nullptr;
    unsigned xe_total = 0;           // remote-tile ends counted in *xe_done so far (mod 2**32)
    // diagnostics (timing class PAMG_K_HALO_EARLY enabled): events at the last early-exchange call's launch
    // start, exchange start (the signal seen), exchange end and launch end
    hipEvent_t xe_ev[4] = {nullptr, nullptr, nullptr, nullptr};
    bool xe_ev_valid = false;
    int cus = 0;                     // compute units of the device
    // op = 1 on a partition: the coarsest level agglomerated (pamg_api.cpp agg_*). `agg` is a
    // replica handle holding only level L of the WHOLE mesh, un_eles renumbered so that every rank's are one
    // block (agg_off[r] .. agg_off[r + 1]); it shares this handle's stream. Each cycle gathers the ranks' level-L
    // RHS into it and every rank runs the single-domain coarsest calls (the persistent chain) on its own copy.
    pamg_handle *agg = nullptr;
    std::vector<int> agg_off;
    bool coarse_only = false;        // this handle is such a replica: levels below L are not allocated
    bool borrowed_stream = false;    // `stream` belongs to another handle (the replica's parent)
    pamg_handle *tparent = nullptr;  // the replica's timing spans and fallback counts go to its parent's Timing
};

// ---- setup (pamg_setup.cpp) ----
namespace pamg {
void get_str_info(int n_split, int ele, int *irow, int *ipos, int *orientation);
void element_conversion(int fin[4], int coarse_ele, int i_split);
void loc_surf_ele(int n, std::vector<int> &surf);
void get_splitting(const double *un_x, int n_split, int str_ele, double str_x[3][2]);
// storage positions of every level (see Level::pos): levels 1..L of a split n_split
void hier_positions(int n_split, int L, std::vector<int> pos[]);
// D0 (optional, 3): get_diagonal's rdt ml_i + Kd_ii + 0.0 (:481-486)
void level_stencil(const double *X, int i_split, double k, double dt, double omega, double *rec, double *D0 = nullptr);
// M == c [[2,1,1],[1,2,1],[1,1,2]] bit for bit (the form the smoother kernels evaluate)
bool mass_is_p1_midpoint(const double *rec);
int build_halo(pamg_handle *h, int l, const double *Xg, const int *neig, const int *fneig, const int *dir);
// face-coupled operator tables of level l (Level::fnb / fface / fsx, host copies returned)
// fface record per (un_ele, level): w_in[3] | w_b[3] | D0[3] | pad[3] | omega / D[8][3] -- D of a
// sub-element whose faces are inner (bit fi of the pattern) or across an un_ele face, accumulated in
// the oracle's face order (face_terms), divided on the host (IEEE: bitwise the device's division)
constexpr int kFaceStride = 36, kFaceWD = 12;
int build_face(pamg_handle *h, int l, const double *Xg, const int *neig, const int *fneig, const int *dir,
               std::vector<int4> &fnb, std::vector<double> &fface, std::vector<int> &fsx);
}  // namespace pamg

// ---- kernels (pamg_kernels.hip) ----
namespace pamg {
hipError_t launch_smooth(hipStream_t s, const Level &L, const double *src, int sweeps, int solver,
                         double rdt, double omega, double *tov, double *tovo);
hipError_t launch_residual(hipStream_t s, const Level &L, double rdt, bool neg = false);
// corrected cycle: fine.T += P coarse.T (P1 interpolation weights of splitting.F90:59-88)
hipError_t launch_interp_add(hipStream_t s, const Level &fine, const Level &coarse);
hipError_t launch_restrict(hipStream_t s, const Level &fine, const Level &coarse, int U, double *out = nullptr);
hipError_t launch_prolong(hipStream_t s, const Level &fine, const Level &coarse, bool write_tnn);
// start_of_step: 0 RHS from told; 1 told := tnew_nonlin := tnew first; 2 told := tnew first
// told_halo: with start_of_step, also write the compact told copy of the halo (launch_told_halo)
// RHS = rdt M told + s' with s' from L.SRC (launch_source)
hipError_t launch_rhs(hipStream_t s, const Level &L, double rdt, int start_of_step, bool told_halo = false);
// s' of level 1 into L.SRC (once, at upload): the source term of get_RHS from the geometry
hipError_t launch_source(hipStream_t s, const Level &L, const double *geo1, double k);
hipError_t launch_halo_unpack(hipStream_t s, const Level &L, double *tov, double *tovo);
// the tnew words of one cycle of the resident call's ring exchange (3 per entry, d_recv3) into t_overlap
hipError_t launch_halo_unpack3(hipStream_t s, const Level &L, double *tov);
hipError_t launch_copy(hipStream_t s, const double *src, double *dst, int64_t n);
hipError_t launch_told_halo(hipStream_t s, const Level &L, int U);
// from_told: read told from the TOLD planes and also write the compact told copy
// (launch_told_halo's words) instead of reading that copy
hipError_t launch_overlap_static(hipStream_t s, const Level &L, int U, double *tov, double *tovo,
                                 double *send = nullptr, bool from_told = false);
// fused V-cycle (pamg_vcycle.hip); lv is the handle's 1-based level array
bool vcycle_fusable(const Level *lv, int L, int n_split, int solver, int halo_mode, int n_smooth);
// levels 2..L; the level-2 RHS is taken from rhsn2 (level 2's RHSN or RHSN_alt)
// stores a pipelined V-cycle launch may skip (pamg_vcycle.hip, kKeep*)
constexpr int PAMG_KEEP_L1 = 1, PAMG_KEEP_COARSE = 2, PAMG_KEEP_HALO = 4, PAMG_KEEP_ALL = 7;
// RHSF launches (the first level-1 launch of a pamg_run step, which starts the step): store
// told and write the halo words that are constant within the step (k_overlap_static's) --
// skipped when the next step overwrites them unread
constexpr int PAMG_KEEP_TOLD = 8;
// [ua, ub): the un_eles a launch covers (ub < 0: all of them); bounds multiples of
// vcycle_tile_un_eles (ub may be U)
hipError_t launch_vcycle_coarse(hipStream_t s, const Level *lv, int L, int U, int n_split, int n_smooth,
                                int n_coarse, double rdt, double *tov, double *tovo, const double *rhsn2, int ua = 0,
                                int ub = -1, int keep = PAMG_KEEP_ALL);
int vcycle_tile_un_eles(int n_split);
bool vcycle_rhsf_supported(int n_split);
// level 1; its remote halo words packed into send1 (one of level 1's two send buffers), the
// restriction of its residual into rhsn2
// pipe: the same launch also runs the coarse levels of the next cycle (L >= 2; level 2's RHS
// from LDS, rhsn2 unused); keep: which of its dead-until-final stores it makes
// (PAMG_KEEP_*, pamg_vcycle.hip)
// rhsf (pipe only): the launch also starts the time step (told := tnew, RHS = rdt M told + s');
// with keep & PAMG_KEEP_TOLD it stores told and writes the step's constant halo words, the told
// halves of the send entries into both send1 and send_b
hipError_t launch_vcycle_fine(hipStream_t s, const Level *lv, int L, int U, int n_split, int n_smooth,
                              int n_coarse, double rdt, double *tov, double *tovo, double *send1, double *rhsn2,
                              bool pipe = false, int keep = PAMG_KEEP_ALL, int ua = 0, int ub = -1,
                              bool rhsf = false, double *send_b = nullptr);
// the resident form: all `cycles` cycles of a call in one launch, every level's state on-chip
// between them (first coarse cycle included: level 2's RHS from rhsn2); the final-cycle
// stores as keep says; rhsf: the launch starts the time step (as launch_vcycle_fine's)
// steps > 1 (rhsf): a whole pamg_run -- `steps` time steps of `cycles` cycles, each step starting
// with told := tnew and its RHS -- in one launch (vcycle_resident_run_supported)
// the early per-call exchange (pamg_api.cpp vcycle_fused): the workgroups take the tiles in tile_map's
// order (remote tiles first); each tile with a face on another rank counts its end in *done once its send
// words are written through, and the one whose count reaches `target` (the running total of remote-tile
// ends, mod 2**32: the counter is never reset) adds 1 to *sig
struct EarlyXc {
    const int *tile_map;
    unsigned *done;
    unsigned target;
    unsigned long long *sig;
};
hipError_t launch_vcycle_resident(hipStream_t s, const Level *lv, int L, int U, int n_split, int n_smooth,
                                  int n_coarse, double rdt, double *tov, double *tovo, double *send1, double *rhsn2,
                                  int keep, bool rhsf, double *send_b, int cycles, int steps = 1,
                                  const EarlyXc *xe = nullptr);
// per level-1 tile of the resident launch: does it hold a face whose neighbour is on another rank
void vcycle_remote_tiles(const Level &L1, int U, int n_split, std::vector<char> &remote);
// the resident call with an exchange after every cycle (halo_exchange = 1): cycle c < cycles - 1
// packs its remote halo words (3 per entry) into ring + c ring_stride and, once every workgroup has,
// adds 1 to *xc_sig (xc_done: cycles - 1 zeroed counters); the last cycle is the plain resident call's
hipError_t launch_vcycle_resident_xc(hipStream_t s, const Level *lv, int L, int U, int n_split, int n_smooth,
                                     int n_coarse, double rdt, double *tov, double *tovo, double *send1,
                                     double *rhsn2, int keep, int cycles, double *ring, int64_t ring_stride,
                                     unsigned *xc_done, unsigned long long *xc_sig);
bool vcycle_resident_supported(int n_split, int L);
// the corrected V-cycle (pamg_params.cycle = 1) as one resident launch per call (k_vc_corr): `cycles`
// cycles, every level of a tile on-chip, the final state and level 1's halo words stored at the end
// (keep & PAMG_KEEP_HALO; remote words packed into send1); the state is the per-step sequence's
hipError_t launch_vcycle_corrected(hipStream_t s, const Level *lv, int L, int U, int n_split, int n_smooth,
                                   int n_coarse, double rdt, double *tov, double *tovo, double *send1, double *rhsn2,
                                   int keep, int cycles);
bool vcycle_corrected_supported(int n_split, int L);
bool vcycle_resident_run_supported(int n_split, int L);
hipError_t launch_restrict_residual(hipStream_t s, const Level &fine, const Level &coarse, double rdt);
hipError_t launch_to_soa(hipStream_t s, const Level &L, const double *aos, double *soa);
// FINDInv (matrix_inversion.F90:50-148) batched, n <= 8, column-major (n, n, nb)
hipError_t launch_block_inverse(hipStream_t s, int n, int64_t nb, const double *A, double *inv, int *err);
// A_e = (1/dt) M + Kd per un_ele of level L and its FINDInv inverse (9 fp64 per un_ele)
hipError_t launch_block_ops(hipStream_t s, const Level &L, int U, double rdt, double *Ainv, int *err);
// direct local solve of level L: tnew = tnew_nonlin = A_e^-1 RHS
hipError_t launch_block_solve(hipStream_t s, const Level &L, const double *Ainv);
hipError_t launch_to_aos(hipStream_t s, const Level &L, const double *soa, double *aos);
hipError_t launch_build_blocks(hipStream_t s, const Level &L, double rdt);
size_t asm_blocks_doubles(const Level &L);   // the size of Level::blocks (launch_build_blocks' layout)
// face-coupled operator (pamg_face.hip): the halo words of level L from its tnew (copy: tnew :=
// tnew_nonlin first, the sweep start :550); one sweep (mode 0 up sub-elements, 1 down ones --
// red-black Gauss-Seidel in place on tnew_nonlin -- 2 Jacobi from tnew); the residual A tnew - RHS
// (neg: RHS - A tnew); level1: the domain-boundary values enter (coarse levels: zero)
hipError_t launch_face_halo(hipStream_t s, const Level &L, double *tov, double *tovo, bool copy);
// the same words as launch_face_halo(copy = false), from tnew, over the sub-elements that have them
hipError_t launch_face_words(hipStream_t s, const Level &L, int U, double *tov, double *tovo);
hipError_t launch_face_sweep(hipStream_t s, const Level &L, const double *tov, int mode, bool level1, double rdt,
                             double omega, int slots);
hipError_t launch_face_residual(hipStream_t s, const Level &L, const double *tov, bool neg, bool level1, double rdt,
                                int slots);
// one whole face-operator sweep in one launch (copy, both colours or Jacobi, the next sweep's halo
// words into tout; single domain, un_eles of at most 4096 sub-elements)
bool face_sweep_fusable(const Level &L);
// store: 0 tnew_nonlin; 1 tnew_nonlin and tnew (the sweep's start); 2 tnew := the result only (the
// last executed sweep of a call whose final sweep is dead); bc: the call's first sweep (its next-halo
// words include the boundary words of the other snapshot buffer)
hipError_t launch_face_sweep_fused(hipStream_t s, const Level &L, const double *tin, double *tout, double *tovo,
                                   bool rb, bool level1, double rdt, double omega, int slots, int store, bool bc, bool from_T = false,
                                   double *res = nullptr);
// k_face_tile's levels (one tile per un_ele); their first sweep can also write get_residual (res)
bool face_tile_shape(const Level &L);
// K = 1 or 2 sweeps in one launch from the iterate `in` (read-only: the neighbours' halo values are read
// from it, the second sweep's computed in the launch); res 1 / 2: get_residual into L.RES of the start
// iterate / the iterate after the first sweep; out_pre / out_mid / out_end (any may be null, none `in`):
// the start iterate, the iterate after sweep 1, after the last sweep
// k_face_pp's folds of the coarse level (launch_face_pp): rhsc -- the pass's residual restricted into this buffer (the
// coarse level's layout), res_store -- the residual itself stored too (L.RES), interp -- the coarse level's T
// prolonged and added to every value the pass loads
struct PPCoarse {
    const Level *coarse = nullptr;
    double *rhsc = nullptr;
    bool res_store = true;
    bool interp = false;
};
hipError_t launch_face_pp(hipStream_t s, const Level &L, int K, const double *in, double *out_pre, double *out_mid,
                          double *out_end, bool rb, bool level1, double rdt, int res, double *out_end2 = nullptr,
                          const PPCoarse *pc = nullptr);
// guard: the workgroups check that they are all resident before touching the state; if not, none does and
// the launch counts an abort in tmo[3] (tmo[1..2] the guard's own words) -- the host runs the call another way
// the persistent chain of one face-operator smoother call (single domain; face_chain_fits): `run` of
// the call's `total` sweeps in one launch, the iterate in LDS, the halo handed over between
// workgroups inside the launch; store 1: tnew (the last sweep's start) and tnew_nonlin, 2: tnew :=
// the result (dead last sweep)
bool face_chain_fits(int nsub, int U, int cus);
// the wavefront form of one smoother call (k_face_wave, levels of 256 / 1,024 / 4,096 sub-elements
// per un_ele): un_eles claimed in the ticket order `order`, flags = U per-un_ele words + the ticket
// counter (zeroed here); g0 / g1 the tagged halo granules of odd / even sweeps (2 words per t_overlap
// double), tag0 + s the tag of sweep s (never reused: the host advances it past every launch's tags);
// grid = co-resident workgroups
bool face_wave_shape(const Level &L);
int face_wave_grid(const Level &L, bool rb, int cus);
hipError_t launch_face_wave(hipStream_t s, const Level &L, int U, int grid, double *tov, double *tov_b, double *tovo,
                            unsigned long long *g0, unsigned long long *g1, unsigned tag0, unsigned *flags,
                            const int *order, unsigned *tmo, int run, int total, int store, bool rb, bool level1,
                            double rdt, int slots, bool from_T = false);
int face_chain_per_wg(int nsub, int U, int cus);
// a chain launch's gate report (pamg_face.hip chain_leave; gate null: none)
constexpr unsigned long long kGateRing = 1024;
struct ChainGate {
    unsigned long long *gate = nullptr, *stat = nullptr;
    unsigned long long seq = 0;
};
hipError_t launch_face_chain(hipStream_t s, const Level &L, int U, int cus, double *tov, double *tov_b, double *tovo,
                             unsigned *flags, const int *nb_off, const int *nb_list, unsigned *tmo, int run, int total,
                             int store, bool rb, bool level1, double rdt, double omega, int slots, bool from_T = false,
                             unsigned f0 = 0, int guard = 0, ChainGate G = ChainGate());
hipError_t launch_sweep_assembled(hipStream_t s, const Level &L, double *out, double rdt);
hipError_t launch_sweep_stencil(hipStream_t s, const Level &L, double *out, double rdt);
}  // namespace pamg
