// C-ABI of libpamg: handle, setup, state transfer, the hot-path entry points
// (one per reference call site) and the V-cycle driver of
// transport_tri_semi.F90:299-381.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "pamg_internal.h"

using namespace pamg;

namespace pamg {
// Single-process device-copy transport (pamg_comm_local_group): n partition handles of one
// owner map, each driven by its own host thread like one process per rank. The exchange is
// the RCCL one with ncclSend / ncclRecv replaced by device-to-device copies between the
// handles: a rank posts its packed send words (pointer + an event recorded after the
// packing) to every peer, pulls each peer's words for it into its own receive buffer behind
// that peer's event, and then waits, before it may repack, until every peer has issued its
// reads of its words (the send completion of ncclSend). Posts carry a per-pair sequence
// number, so ranks meet exchange by exchange as grouped send/recv calls do.
struct LocalGroup {
    struct Post { long seq = 0; const double *ptr = nullptr; hipEvent_t ev = nullptr; int64_t pitch = 0; };
    int n = 0;
    std::mutex mu;
    std::condition_variable cv;
    std::vector<Post> ready, done;   // [src * n + dst]
    int refs = 0;
};
struct Comm {
    ncclComm_t nccl = nullptr;
    LocalGroup *local = nullptr;
    std::vector<long> seq;           // per peer index (level 1's plan): exchanges completed
    hipEvent_t ev_ready = nullptr, ev_done = nullptr;
};
}  // namespace pamg

#define HIPCHK(h, expr)                                                                   \
    do {                                                                                  \
        hipError_t e_ = (expr);                                                           \
        if (e_ != hipSuccess) {                                                           \
            (h)->err = std::string(#expr) + ": " + hipGetErrorString(e_);                 \
            return PAMG_ERR_HIP;                                                          \
        }                                                                                 \
    } while (0)

#define NCCLCHK(h, expr)                                                                  \
    do {                                                                                  \
        ncclResult_t r_ = (expr);                                                         \
        if (r_ != ncclSuccess) {                                                          \
            (h)->err = std::string(#expr) + ": " + ncclGetErrorString(r_);                \
            return PAMG_ERR_COMM;                                                         \
        }                                                                                 \
    } while (0)

#define CHK(expr)                    \
    do {                             \
        int rc_ = (expr);            \
        if (rc_ != PAMG_OK) return rc_; \
    } while (0)

namespace {

template <class T>
int dev_alloc(pamg_handle *h, T **p, size_t count) {
    *p = nullptr;
    if (count == 0) return PAMG_OK;
    HIPCHK(h, hipMalloc((void **)p, count * sizeof(T)));
    return PAMG_OK;
}

// every setup transfer runs on the handle's stream: its streams are non-blocking, so work on
// them is not ordered against the null stream a blocking hipMemcpy uses (a memset queued on
// h->stream could land after such a copy)
int face_gates_drain(pamg_handle *h);   // (a host wait on the handle's stream first reads its chain gates back)

template <class T>
int dev_upload(pamg_handle *h, T **p, const std::vector<T> &v) {
    CHK(dev_alloc(h, p, v.size()));
    if (!v.empty()) {
        CHK(face_gates_drain(h));
        HIPCHK(h, hipMemcpyAsync(*p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice, h->stream));
        HIPCHK(h, hipStreamSynchronize(h->stream));   // v may be freed on return
    }
    return PAMG_OK;
}

void dev_free(void *p) {
    if (p) (void)hipFree(p);
}

int check_level(pamg_handle *h, int l) {
    if (!h->mesh_ready) { h->err = "mesh not uploaded"; return PAMG_ERR_STATE; }
    if (l < 1 || l > h->p.multi_levels) { h->err = "level out of range"; return PAMG_ERR_ARG; }
    return PAMG_OK;
}

// ---- timing -------------------------------------------------------------
hipEvent_t take_event(pamg_handle *h) {
    auto &pool = h->timing.pool;
    if (!pool.empty()) { hipEvent_t e = pool.back(); pool.pop_back(); return e; }
    hipEvent_t e = nullptr;
    (void)hipEventCreate(&e);
    return e;
}

// an event pair around the work issued in a scope, on stream s, when its timing class is enabled (one in
// `stride` of its spans). (Events recorded in the resident launch's own dispatch packet, hipExtLaunchKernel,
// measured no cheaper than the marker pair: profiles/r05_a_shape_probe.txt, r05_c_events_ab.txt; removed.)
struct Span {
    pamg_handle *h; int kid; double bytes; hipStream_t s; hipEvent_t a = nullptr, b = nullptr;
    Span(pamg_handle *h_, int kid_, double bytes_, hipStream_t s_ = nullptr)
        : h(h_->tparent ? h_->tparent : h_), kid(kid_), bytes(bytes_), s(s_ ? s_ : h_->stream) {
        if ((h->timing.mask & (1u << kid)) && h->timing.seq[kid]++ % h->timing.stride == 0) {
            a = take_event(h);
            (void)hipEventRecord(a, s);
        }
    }
    ~Span() {
        if (!a) return;
        b = take_event(h);
        (void)hipEventRecord(b, s);
        h->timing.pending.push_back(Timing::Rec{kid, a, b, bytes});
    }
};

int settle(pamg_handle *h);
int sync_stream(pamg_handle *h, hipStream_t s);
int drain_timing(pamg_handle *h) {
    auto &T = h->timing;
    if (T.pending.empty()) return PAMG_OK;
    // spans may sit on the comm stream (the exchange spans, the early exchange's): the stream joins every
    // exchange in flight first, and the comm stream is drained too, so no event pair is read before it ran
    CHK(settle(h));
    CHK(sync_stream(h, h->stream));
    CHK(sync_stream(h, h->stream_comm));
    for (auto &r : T.pending) {
        float ms = 0.f;
        HIPCHK(h, hipEventElapsedTime(&ms, r.a, r.b));
        T.ms[r.kid] += ms;
        T.count[r.kid] += 1;
        T.bytes[r.kid] += r.bytes;
        T.pool.push_back(r.a);
        T.pool.push_back(r.b);
    }
    T.pending.clear();
    return PAMG_OK;
}

// ---- scratch ------------------------------------------------------------
int ensure_scratch(pamg_handle *h, size_t bytes) {
    if (h->scratch_bytes >= bytes) return PAMG_OK;
    CHK(face_gates_drain(h));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    dev_free(h->scratch);
    h->scratch = nullptr;
    h->scratch_bytes = 0;
    HIPCHK(h, hipMalloc((void **)&h->scratch, bytes));
    h->scratch_bytes = bytes;
    return PAMG_OK;
}

double *field_ptr(pamg_handle *h, int l, int what) {
    Level &L = h->lv[l];
    switch (what) {
        case PAMG_TNEW: return L.T;
        case PAMG_TOLD: return L.TOLD;
        case PAMG_RHS: return L.RHS;
        case PAMG_RESIDUAL: return L.RES;
        case PAMG_TNEW_NONLIN: return L.TNN;
        case PAMG_SOURCE: return L.SRC;   // level 1 only (null elsewhere)
    }
    return nullptr;
}

// ---- halo exchange --------------------------------------------------------
// The halo words of a smoother call are written by the smoother kernel itself
// (local neighbours and boundary values into t_overlap, remote neighbours into
// the packed send buffer); what remains here is the exchange with other ranks.
// pamg_comm_local_group transport: the grouped send/recv below as device copies between the
// partition handles of one process (LocalGroup)
int local_timeout_s() {
    const char *e = getenv("PAMG_COMM_TIMEOUT_S");
    const int t = e ? atoi(e) : 120;
    return t > 0 ? t : 120;
}

// Bounded RCCL waits. A grouped send/recv that answers ncclInProgress is polled here for at
// most PAMG_COMM_TIMEOUT_S (default 120 s, the local group's exchange bound), and every host wait for a stream
// that carries exchanges is bounded the same way (sync_stream); on the bound or an error the communicator is
// aborted, so a rank that stops issuing exchanges ends its peers' calls with PAMG_ERR_COMM instead of hanging
// them. The communicator's initialisation cannot be bounded from here: RCCL 2.27's bootstrap waits for every
// rank, and a non-blocking communicator (ncclConfig_t::blocking = 0) blocked inside ncclCommInitRankConfig
// itself, while a blocking init left on a helper thread faults the process at exit
// (profiles/r06_rccl_init_probe.txt). The caller's launcher bounds it (bench.py: a gloo barrier with a timeout
// right before pamg_comm_init), and the communicator stays blocking.
int nccl_settle(ncclComm_t c, ncclResult_t r, int limit_s, std::string &err, const char *what) {
    const auto t0 = std::chrono::steady_clock::now();
    while (r == ncclInProgress) {
        if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(limit_s)) {
            err = std::string(what) + ": not complete within " + std::to_string(limit_s) +
                  " s (PAMG_COMM_TIMEOUT_S); a peer rank did not join or stopped";
            return PAMG_ERR_COMM;
        }
        std::this_thread::sleep_for(std::chrono::microseconds(50));
        if (ncclCommGetAsyncError(c, &r) != ncclSuccess) r = ncclSystemError;
    }
    if (r != ncclSuccess) {
        err = std::string(what) + ": " + ncclGetErrorString(r);
        return PAMG_ERR_COMM;
    }
    return PAMG_OK;
}

// a grouped send/recv's end: polled to completion of its enqueueing; the communicator aborted on failure
int nccl_group_end(pamg_handle *h) {
    const ncclResult_t r = ncclGroupEnd();
    const int rc = nccl_settle(h->comm->nccl, r, local_timeout_s(), h->err, "ncclGroupEnd (halo exchange)");
    if (rc != PAMG_OK) {
        (void)ncclCommAbort(h->comm->nccl);
        h->comm->nccl = nullptr;
    }
    return rc;
}

// ncclSend / ncclRecv inside a group only enqueue (a non-blocking communicator may answer ncclInProgress)
#define NCCLQ(h, expr)                                                                    \
    do {                                                                                  \
        ncclResult_t r_ = (expr);                                                         \
        if (r_ != ncclSuccess && r_ != ncclInProgress) {                                  \
            (void)ncclGroupEnd();                                                         \
            (h)->err = std::string(#expr) + ": " + ncclGetErrorString(r_);                \
            return PAMG_ERR_COMM;                                                         \
        }                                                                                 \
    } while (0)

// w words per entry (6: tnew and told; 3: the tnew words of the resident call's ring), into recv
int exchange_local(pamg_handle *h, int l, const double *send, hipStream_t st, int w, double *recv) {
    Comm &C = *h->comm;
    LocalGroup &G = *C.local;
    const HaloPlan &P = h->lv[l].halo;
    const int me = h->rank, np = (int)P.peers.size();
    std::vector<LocalGroup::Post> got(np);
    auto wait_posts = [&](std::vector<LocalGroup::Post> &box, const char *what) -> int {
        std::unique_lock<std::mutex> lk(G.mu);
        for (int q = 0; q < np; ++q) {
            const int peer = P.peers[q];
            const long want = C.seq[peer] + 1;
            LocalGroup::Post &b = box[(size_t)peer * G.n + me];
            if (!G.cv.wait_for(lk, std::chrono::seconds(local_timeout_s()), [&] { return b.seq >= want; })) {
                h->err = "local halo exchange: rank " + std::to_string(me) + " timed out waiting for rank " +
                         std::to_string(peer) + "'s " + what;
                return PAMG_ERR_COMM;
            }
            if (b.seq != want) { h->err = "local halo exchange: sequence mismatch"; return PAMG_ERR_COMM; }
            got[q] = b;
        }
        return PAMG_OK;
    };
    // 1. post the packed words, pull the peers' words for this rank behind their events
    HIPCHK(h, hipEventRecord(C.ev_ready, st));
    {
        std::lock_guard<std::mutex> lk(G.mu);
        for (int q = 0; q < np; ++q) {
            const int peer = P.peers[q];
            G.ready[(size_t)me * G.n + peer] = {C.seq[peer] + 1, send + w * (size_t)P.send_peer_off[q], C.ev_ready};
        }
    }
    G.cv.notify_all();
    CHK(wait_posts(G.ready, "send words"));
    for (int q = 0; q < np; ++q) {
        const size_t nr = (size_t)(P.recv_peer_off[q + 1] - P.recv_peer_off[q]);
        HIPCHK(h, hipStreamWaitEvent(st, got[q].ev, 0));
        if (nr)
            HIPCHK(h, hipMemcpyAsync(recv + w * (size_t)P.recv_peer_off[q], got[q].ptr, w * nr * sizeof(double),
                                     hipMemcpyDeviceToDevice, st));
    }
    // 2. this rank's reads are issued; its send words may be repacked once every peer's are
    HIPCHK(h, hipEventRecord(C.ev_done, st));
    {
        std::lock_guard<std::mutex> lk(G.mu);
        for (int q = 0; q < np; ++q) {
            const int peer = P.peers[q];
            G.done[(size_t)me * G.n + peer] = {C.seq[peer] + 1, nullptr, C.ev_done};
        }
    }
    G.cv.notify_all();
    CHK(wait_posts(G.done, "receive completion"));
    for (int q = 0; q < np; ++q) {
        HIPCHK(h, hipStreamWaitEvent(st, got[q].ev, 0));
        C.seq[P.peers[q]] += 1;
    }
    return PAMG_OK;
}

// dst: the t_overlap buffer the received words go into (h->tov unless a face call's other snapshot buffer)
int exchange(pamg_handle *h, int l, int buf, hipStream_t st, double *dst = nullptr) {
    Level &L = h->lv[l];
    const HaloPlan &P = L.halo;
    const double *send = P.send_buf(buf);
    if (!dst) dst = h->tov;
    Span sp(h, PAMG_K_HALO, 2.0 * 48.0 * (double)(P.remote.size() + P.recv_dst.size()), st);
    if (h->comm->local) {
        CHK(exchange_local(h, l, send, st, 6, P.d_recv));
        HIPCHK(h, launch_halo_unpack(st, L, dst, h->tovo));
        return PAMG_OK;
    }
    NCCLCHK(h, ncclGroupStart());
    for (size_t q = 0; q < P.peers.size(); ++q) {
        const int peer = P.peers[q];
        const size_t ns = (size_t)(P.send_peer_off[q + 1] - P.send_peer_off[q]);
        const size_t nr = (size_t)(P.recv_peer_off[q + 1] - P.recv_peer_off[q]);
        if (ns) NCCLQ(h, ncclSend(send + 6 * (size_t)P.send_peer_off[q], 6 * ns, ncclDouble, peer, h->comm->nccl, st));
        if (nr) NCCLQ(h, ncclRecv(P.d_recv + 6 * (size_t)P.recv_peer_off[q], 6 * nr, ncclDouble, peer,
                                  h->comm->nccl, st));
    }
    CHK(nccl_group_end(h));
    HIPCHK(h, launch_halo_unpack(st, L, dst, h->tovo));
    return PAMG_OK;
}

// the tnew words of cycle c of a resident call with halo_exchange = 1 (level 1's ring, 3 words per
// entry; the told words do not change within a time step and travel with the last cycle's exchange)
int exchange_ring(pamg_handle *h, int c, hipStream_t st) {
    Level &L = h->lv[1];
    const HaloPlan &P = L.halo;
    const double *send = P.d_ring + (size_t)c * 3 * P.remote.size();
    Span sp(h, PAMG_K_HALO, 2.0 * 24.0 * (double)(P.remote.size() + P.recv_dst.size()), st);
    if (h->comm->local) {
        CHK(exchange_local(h, 1, send, st, 3, P.d_recv3));
        HIPCHK(h, launch_halo_unpack3(st, L, h->tov));
        return PAMG_OK;
    }
    NCCLCHK(h, ncclGroupStart());
    for (size_t q = 0; q < P.peers.size(); ++q) {
        const int peer = P.peers[q];
        const size_t ns = (size_t)(P.send_peer_off[q + 1] - P.send_peer_off[q]);
        const size_t nr = (size_t)(P.recv_peer_off[q + 1] - P.recv_peer_off[q]);
        if (ns) NCCLQ(h, ncclSend(send + 3 * (size_t)P.send_peer_off[q], 3 * ns, ncclDouble, peer, h->comm->nccl, st));
        if (nr) NCCLQ(h, ncclRecv(P.d_recv3 + 3 * (size_t)P.recv_peer_off[q], 3 * nr, ncclDouble, peer,
                                  h->comm->nccl, st));
    }
    CHK(nccl_group_end(h));
    HIPCHK(h, launch_halo_unpack3(st, L, h->tov));
    return PAMG_OK;
}

int sync_stream(pamg_handle *h, hipStream_t s);

// the ring, counters and signal of a resident call of `cycles` cycles with halo_exchange = 1
int xc_setup(pamg_handle *h, int cycles) {
    HaloPlan &P = h->lv[1].halo;
    const int need = cycles - 1;
    if (P.ring_cap < need) {
        CHK(sync_stream(h, h->stream));
        CHK(sync_stream(h, h->stream_comm));
        dev_free(P.d_ring);
        P.d_ring = nullptr;
        P.ring_cap = 0;
        CHK(dev_alloc(h, &P.d_ring, (size_t)need * 3 * P.remote.size()));
        P.ring_cap = need;
    }
    if (!P.d_recv3 && !P.recv_dst.empty()) CHK(dev_alloc(h, &P.d_recv3, 3 * P.recv_dst.size()));
    if (h->xc_cap < need) {
        CHK(sync_stream(h, h->stream));
        dev_free(h->xc_done);
        h->xc_done = nullptr;
        h->xc_cap = 0;
        CHK(dev_alloc(h, &h->xc_done, (size_t)need));
        h->xc_cap = need;
    }
    if (!h->xc_sig) {
        // the comm stream waits on it (hipStreamWaitValue64): HIP's signal memory
        HIPCHK(h, hipExtMallocWithFlags((void **)&h->xc_sig, sizeof(unsigned long long), hipMallocSignalMemory));
        unsigned long long v = 0;
        HIPCHK(h, hipMemcpy(&v, h->xc_sig, sizeof v, hipMemcpyDeviceToHost));
        h->xc_sig_base = v;
    }
    return PAMG_OK;
}

// the early per-call exchange of the resident call: the tile order with the tiles that hold a remote
// face first (they then run in the launch's first round of workgroups, and the exchange of their words
// overlaps the rounds after it), the counter and the signal. PAMG_EARLY_XC=0 turns it off (A/B runs)
int xe_setup(pamg_handle *h) {
    if (h->xe_nremote < 0) {
        std::vector<char> rem;
        vcycle_remote_tiles(h->lv[1], h->U, h->p.n_split, rem);
        std::vector<int> order;
        order.reserve(rem.size());
        for (size_t b = 0; b < rem.size(); ++b)
            if (rem[b]) order.push_back((int)b);
        const int nr = (int)order.size();
        for (size_t b = 0; b < rem.size(); ++b)
            if (!rem[b]) order.push_back((int)b);
        if (nr > 0) CHK(dev_upload(h, &h->xe_map, order));
        h->xe_nremote = nr;
    }
    if (h->xe_nremote > 0 && !h->xe_done) {
        CHK(dev_alloc(h, &h->xe_done, 1));
        HIPCHK(h, hipMemsetAsync(h->xe_done, 0, sizeof(unsigned), h->stream));
        h->xe_total = 0;
    }
    if (h->xe_nremote > 0 && !h->xc_sig) {
        HIPCHK(h, hipExtMallocWithFlags((void **)&h->xc_sig, sizeof(unsigned long long), hipMallocSignalMemory));
        unsigned long long v = 0;
        HIPCHK(h, hipMemcpy(&v, h->xc_sig, sizeof v, hipMemcpyDeviceToHost));
        h->xc_sig_base = v;
    }
    return PAMG_OK;
}


int halo(pamg_handle *h, int l, double *dst = nullptr) {
    const HaloPlan &P = h->lv[l].halo;
    if (h->comm && !P.peers.empty()) {
        h->lv[l].halo.send_cur = 0;   // the per-step kernels pack into the first buffer
        return exchange(h, l, 0, h->stream, dst);
    }
    return PAMG_OK;
}

// fused V-cycle: the exchange of level 1's words packed into `buf` runs on stream_comm,
// overlapped with the next cycle (nothing in a cycle reads t_overlap)
int halo_async(pamg_handle *h, int buf) {
    HaloPlan &P = h->lv[1].halo;
    P.send_cur = buf;
    if (!h->comm || P.peers.empty()) return PAMG_OK;
    HIPCHK(h, hipEventRecord(h->ev_packed, h->stream));
    HIPCHK(h, hipStreamWaitEvent(h->stream_comm, h->ev_packed, 0));
    CHK(exchange(h, 1, buf, h->stream_comm));
    HIPCHK(h, hipEventRecord(h->ev_sent[buf], h->stream_comm));
    h->sent_pending[buf] = true;
    return PAMG_OK;
}

// `stream` continues after every exchange in flight
int join_comm(pamg_handle *h) {
    for (int b = 0; b < 2; ++b)
        if (h->sent_pending[b]) {
            HIPCHK(h, hipStreamWaitEvent(h->stream, h->ev_sent[b], 0));
            h->sent_pending[b] = false;
        }
    return PAMG_OK;
}

// the entry of a call that may read or write what an exchange still in flight touches (the send and receive
// buffers, t_overlap, t_overlap_old): its work waits for the exchange (the resident call's early exchange is
// not joined when the call returns, vcycle_fused). A gated chain launch still unread also blocks the stream
// until the host reads its report (face_gates_drain): every entry reads them first, so no later host wait or
// implicit device synchronisation (hipFree) can wait on a gate that only this thread would open
int settle(pamg_handle *h) {
    CHK(face_gates_drain(h));
    return h->comm ? join_comm(h) : PAMG_OK;
}

// RCCL's asynchronous error state (polled at the ends of the hot-path calls): a
// failed peer or link is reported as PAMG_ERR_COMM instead of a hang in the next exchange
int comm_error(pamg_handle *h) {
    if (!h->comm || !h->comm->nccl) return PAMG_OK;
    ncclResult_t r = ncclSuccess;
    NCCLCHK(h, ncclCommGetAsyncError(h->comm->nccl, &r));
    if (r != ncclSuccess && r != ncclInProgress) {
        h->err = std::string("RCCL asynchronous error: ") + ncclGetErrorString(r);
        (void)ncclCommAbort(h->comm->nccl);
        h->comm->nccl = nullptr;
        return PAMG_ERR_COMM;
    }
    return PAMG_OK;
}

// stream synchronisation that keeps polling RCCL's error state: a rank whose peer failed
// returns PAMG_ERR_COMM (communicator aborted) instead of waiting on a receive that never
// completes; PAMG_COMM_TIMEOUT_S, when set, also bounds the wait. The device-copy transport
// (pamg_comm_local_group) is polled the same way with its exchange bound (PAMG_COMM_TIMEOUT_S,
// default 120 s): its resident call's comm stream waits on a device signal (hipStreamWaitValue64)
// that a faulted or stopped launch would never raise. The poll spins on hipStreamQuery for the first
// PAMG_SYNC_SPIN_MS (default 5 ms; the communicator checked every 256th query), then sleeps 20 us
// between queries and checks the communicator every 16th. A sleep of 20 us lasts ~60 us or more (the
// kernel's timer slack): with the sleeping poll from the start, a rank's 20-cycle call at config 4's
// N = 8 shape (1,024 un_eles, an RCCL self-peer exchange) took 233.7 us against 169.2 us without a
// communicator, its exchange hidden behind the launch (profiles/r05_c_xe_probe.txt)
int sync_stream(pamg_handle *h, hipStream_t s) {
    if (h->tparent) {   // a coarsest-level replica waits as its partition does (the same stream, its exchanges)
        const int rc = sync_stream(h->tparent, s);
        if (rc != PAMG_OK) h->err = h->tparent->err;
        return rc;
    }
    CHK(face_gates_drain(h));
    if (!h->comm || (!h->comm->nccl && !h->comm->local)) {
        HIPCHK(h, hipStreamSynchronize(s));
        return PAMG_OK;
    }
    // PAMG_COMM_TIMEOUT_S (default 120 s) on both transports: a peer that never issues its side of an exchange
    // ends this rank's wait with PAMG_ERR_COMM (RCCL's error state does not report a missing peer)
    const int limit = local_timeout_s();
    constexpr int spin_ms = 5;
    const auto t0 = std::chrono::steady_clock::now();
    const auto spin_end = t0 + std::chrono::milliseconds(spin_ms);
    for (unsigned i = 0;; ++i) {
        const hipError_t e = hipStreamQuery(s);
        if (e == hipSuccess) return PAMG_OK;
        if (e != hipErrorNotReady) HIPCHK(h, e);
        const auto now = std::chrono::steady_clock::now();
        if (now < spin_end && (i & 255) != 255) continue;
        if ((i & 15) == 15 || now < spin_end) CHK(comm_error(h));
        if (limit > 0 && now - t0 > std::chrono::seconds(limit)) {
            if (h->comm->nccl) {
                h->err = "stream did not drain within PAMG_COMM_TIMEOUT_S; RCCL communicator aborted";
                (void)ncclCommAbort(h->comm->nccl);
                h->comm->nccl = nullptr;
            } else {
                h->err = "stream did not drain within PAMG_COMM_TIMEOUT_S (local-group transport)";
            }
            return PAMG_ERR_COMM;
        }
        if (now >= spin_end) std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
}

// the face-coupled operator's smoother call on a single domain, one launch per sweep
// (k_face_sweep): the halo snapshots alternate between two t_overlap buffers so that a sweep's
// halo words for the next sweep never overwrite the ones it reads; the call's last sweep reads
// h->tov, which therefore holds the words of its start, as after the per-colour sequence.
// dead_last (the fused face V-cycle, vcycle_face_fused): the call's last sweep only produces a
// tnew_nonlin that the cycle overwrites unread (:327, :348, :367) -- it is not run; the sweep before
// it stores its result as tnew (the dead sweep's :550) and writes the dead sweep's :555 words into
// h->tov, so tnew and t_overlap are what the full call leaves.
// the persistent chain (pamg_face.hip k_face_chain) for a smoother call of level l: a single
// domain whose level fits one workgroup per CU (face_chain_fits); PAMG_FACE_CHAIN=0 turns it off
bool face_chain_ok(pamg_handle *h, int l) {
    const char *ev = getenv("PAMG_FACE_CHAIN");   // read per call: tests switch it within a process
    if ((ev && atoi(ev) == 0) || h->nranks != 1 || h->comm || h->neig_local.empty()) return false;
    // the coarsest-level replica of a partition in a local group (pamg_comm_local_group: every rank's handle in
    // one process, on one GPU): the ranks' chains would compete for the same CUs, and an aborted one's fallback
    // (the host's launches on stream_fb) can sit behind another rank's gate in a shared hardware queue -- such a
    // replica runs its calls one launch per sweep (bitwise the chain). One process per GPU keeps the chain.
    if (h->tparent && h->tparent->comm && h->tparent->comm->local) return false;
    if (!h->cus) {
        int n = 0;
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, h->device) != hipSuccess || n <= 0) n = 1;
        h->cus = n;
    }
    return face_chain_fits(h->lv[l].nsub, h->U, h->cus);
}

// its neighbour lists: workgroup w owns un_eles [w k, (w+1) k); its neighbours are the other
// workgroups owning a neighbour of one of them (they write the halo words w reads)
int face_chain_setup(pamg_handle *h, int l) {
    Level &L = h->lv[l];
    if (L.chain_g) return PAMG_OK;
    const int U = h->U, g0 = std::max(1, std::min(h->cus, U)), k = (U + g0 - 1) / g0, G = (U + k - 1) / k;
    std::vector<int> off(1, 0), list;
    for (int w = 0; w < G; ++w) {
        std::vector<int> nb;
        for (int q = w * k; q < std::min(U, (w + 1) * k); ++q)
            for (int f = 0; f < 3; ++f) {
                const int n = h->neig_local[3 * (size_t)q + f];
                if (n >= 0 && n / k != w) nb.push_back(n / k);
            }
        std::sort(nb.begin(), nb.end());
        nb.erase(std::unique(nb.begin(), nb.end()), nb.end());
        list.insert(list.end(), nb.begin(), nb.end());
        off.push_back((int)list.size());
    }
    if (list.empty()) list.push_back(0);
    CHK(dev_upload(h, &L.chain_nb_off, off));
    CHK(dev_upload(h, &L.chain_nb_list, list));
    // the polled words in one block of their own, a multiple of 16 bytes from the allocation's start: one
    // per workgroup (k_face_chain) or per wave of it (k_face_chain_pw, 16 a workgroup)
    L.chain_flag_bytes = ((size_t)G * 16 * sizeof(unsigned) + 15) / 16 * 16;
    CHK(dev_alloc(h, &L.chain_flags, L.chain_flag_bytes / sizeof(unsigned)));
    HIPCHK(h, hipMemsetAsync(L.chain_flags, 0, L.chain_flag_bytes, h->stream));
    L.chain_epoch = 0;
    if (!h->chain_tmo) {
        CHK(dev_alloc(h, &h->chain_tmo, 4));
        HIPCHK(h, hipMemsetAsync(h->chain_tmo, 0, 4 * sizeof(unsigned), h->stream));
    }
    L.chain_g = G;
    return PAMG_OK;
}

// The ticket order of the wavefront calls (k_face_wave): reverse Cuthill-McKee over the local
// un_ele graph (BFS from a pseudo-peripheral un_ele of each component, neighbours by ascending
// degree, reversed), and its band max |pos(u) - pos(v)| over the edges -- untitled8192: 3,754 in
// file order, 63 in this one. A call of `run` sweeps needs (run - 1) band + 1 co-resident
// workgroups to drain (pamg_face.hip k_face_wave).
void rcm_order(const std::vector<int> &neig, int U, std::vector<int> &order, int &band) {
    std::vector<int> deg(U, 0), pos(U, -1);
    for (int u = 0; u < U; ++u)
        for (int f = 0; f < 3; ++f) deg[u] += neig[3 * (size_t)u + f] >= 0;
    order.clear();
    std::vector<int> level(U, -1);
    auto bfs = [&](int r, std::vector<int> &out) {   // breadth-first from r; returns the last level's size
        out.clear();
        out.push_back(r);
        level[r] = 0;
        for (size_t i = 0; i < out.size(); ++i) {
            const int u = out[i];
            int nb[3], n = 0;
            for (int f = 0; f < 3; ++f) {
                const int v = neig[3 * (size_t)u + f];
                if (v >= 0 && level[v] < 0) { level[v] = level[u] + 1; nb[n++] = v; }
            }
            std::sort(nb, nb + n, [&](int a, int b) { return deg[a] != deg[b] ? deg[a] < deg[b] : a < b; });
            for (int k = 0; k < n; ++k) out.push_back(nb[k]);
        }
    };
    std::vector<int> comp;
    for (int s = 0; s < U; ++s) {
        if (pos[s] >= 0) continue;
        // pseudo-peripheral start: repeat BFS from a minimum-degree un_ele of the farthest level
        int r = s;
        for (int it = 0; it < 4; ++it) {
            bfs(r, comp);
            const int last = level[comp.back()];
            int best = comp.back();
            for (int u : comp)
                if (level[u] == last && deg[u] < deg[best]) best = u;
            for (int u : comp) level[u] = -1;
            if (best == r) break;
            r = best;
        }
        bfs(r, comp);
        for (int u : comp) pos[u] = 0;   // mark
        order.insert(order.end(), comp.begin(), comp.end());
    }
    std::reverse(order.begin(), order.end());
    for (int i = 0; i < U; ++i) pos[order[i]] = i;
    band = 0;
    for (int u = 0; u < U; ++u)
        for (int f = 0; f < 3; ++f) {
            const int v = neig[3 * (size_t)u + f];
            if (v >= 0) band = std::max(band, std::abs(pos[u] - pos[v]));
        }
}

int face_wave_setup(pamg_handle *h) {
    if (h->wave_band >= 0) return PAMG_OK;
    std::vector<int> order;
    int band = 0;
    rcm_order(h->neig_local, h->U, order, band);
    CHK(dev_upload(h, &h->wave_order, order));
    CHK(dev_alloc(h, &h->wave_flags, (size_t)h->U + 16));
    const size_t ng = (size_t)h->slots * 3 * std::max(h->U, 1) * 2;   // words per granule buffer
    CHK(dev_alloc(h, &h->wave_gran, 2 * ng));
    HIPCHK(h, hipMemsetAsync(h->wave_gran, 0, 2 * ng * sizeof(unsigned long long), h->stream));
    h->wave_tag = 1;
    if (!h->chain_tmo) {
        CHK(dev_alloc(h, &h->chain_tmo, 4));
        HIPCHK(h, hipMemsetAsync(h->chain_tmo, 0, 4 * sizeof(unsigned), h->stream));
    }
    h->wave_band = band;
    return PAMG_OK;
}

// the wavefront form for a call of `run` executed sweeps on level l, opt-in (PAMG_FACE_WAVE=1): it
// is exact at any occupancy (tagged granules) but measured slower than one launch per sweep on the
// bench mesh (profiles/r03_f_face_forms.txt: its hand-offs wait on memory latency, ~40 us per
// ticket). Returns its grid, 0 when off or when the level's shape or the residency bound rules it out
int face_wave_grid_for(pamg_handle *h, int l, int run) {
    const char *ev = getenv("PAMG_FACE_WAVE");   // read per call: tests switch it within a process
    if (!ev || atoi(ev) == 0 || run < 2 || h->nranks != 1 || h->comm || h->neig_local.empty() || !face_wave_shape(h->lv[l])) return 0;
    if (!h->cus) {
        int n = 0;
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, h->device) != hipSuccess || n <= 0) n = 1;
        h->cus = n;
    }
    if (face_wave_setup(h) != PAMG_OK) return 0;
    const int g = face_wave_grid(h->lv[l], h->p.solver == 3, h->cus);
    // every un_ele resident at once, or the ticket window wide enough for the call's sweeps
    if (g <= 0 || (g < h->U && (int64_t)(run - 1) * h->wave_band + 1 > g)) return 0;
    return g;
}

// the give-up word of the chain's and the wavefront's bounded spins: a call that hit it failed, and
// the state it left was computed from halo words that had not all arrived -- the handle's fields are
// invalid after the error (set them again, or start a new time step from a known tnew). Checked only
// when such a launch ran since the last check (the other op = 1 calls stay asynchronous); the word is
// cleared once reported, so the next call on the handle runs again.
int face_gates_drain(pamg_handle *h);

int face_chain_check(pamg_handle *h) {
    CHK(face_gates_drain(h));
    if (h->agg) {
        const int rc = face_chain_check(h->agg);
        if (rc != PAMG_OK) { h->err = h->agg->err; return rc; }
    }
    if (!h->chain_tmo || !h->chain_pending) return PAMG_OK;
    h->chain_pending = false;
    unsigned v = 0;
    HIPCHK(h, hipMemcpyAsync(&v, h->chain_tmo, sizeof v, hipMemcpyDeviceToHost, h->stream));
    CHK(sync_stream(h, h->stream));
    if (v) {
        HIPCHK(h, hipMemsetAsync(h->chain_tmo, 0, sizeof v, h->stream));
        h->err = "face chain: a workgroup gave up waiting for its neighbours' halo words (the state is invalid)";
        return PAMG_ERR_HIP;
    }
    return PAMG_OK;
}

// a sweep as one launch on LDS tiles (k_face_tile / k_face_sweep) instead of the two colour
// launches (the per-colour kernels remain for the level shapes the tiles do not cover)
bool face_tiles_ok(pamg_handle *h, int l) { return h->p.op == 1 && face_sweep_fusable(h->lv[l]); }

// ... and the whole smoother call with the halo words handed from sweep to sweep on the device
// (face_call): a single domain (a partition exchanges them between sweeps)
// (on a partition too: the words a launch writes for the next sweep -- the remote ones into the send buffer
// -- are exchanged before that sweep, into the snapshot buffer it reads)
bool face_fusable(pamg_handle *h, int l) { return face_tiles_ok(h, l); }

int face_residual(pamg_handle *h, int l, bool neg);

// face_call's executed sweeps as one launch each (from the snapshot the call's halo refresh wrote)
int face_call_sweeps(pamg_handle *h, int l, int sweeps, int run, bool dead_last, bool src_is_T, bool both, bool res_in_sweep) {
    Level &L = h->lv[l];
    const double rdt = 1 / h->p.dt;
    const int kid = (l == 1) ? PAMG_K_SMOOTH_L1 : PAMG_K_SMOOTH;
    double *buf[2] = {h->tov, h->tov_b};
    for (int s = 0; s < run; ++s) {
        const bool fin = s + 1 == run;
        // read tnew_nonlin, RHS; write tnew_nonlin (+ tnew in the last sweep, + the next halo words)
        const int store = fin ? (dead_last ? 2 : 1) : 0;
        const bool r = s == 0 && res_in_sweep;
        if (r) h->rhsn_valid = false;
        Span sp(h, kid, (store == 1 ? 96.0 : 72.0) * (double)L.N + (r ? 24.0 * (double)L.N : 0.0) + 168.0 * h->U);
        HIPCHK(h, launch_face_sweep_fused(h->stream, L, buf[(sweeps - 1 - s) & 1],
                                          s + 1 < sweeps ? buf[(sweeps - 2 - s) & 1] : nullptr, h->tovo,
                                          h->p.solver == 3, l == 1, rdt, h->p.omega, h->slots, store, s == 0,
                                          s == 0 && src_is_T, r ? L.RES : nullptr));
        if (s + 1 < sweeps) CHK(halo(h, l, buf[(sweeps - 2 - s) & 1]));   // the next sweep's remote words
    }
    if (both) HIPCHK(h, launch_copy(h->stream, L.TNN, L.T, 3 * L.pitch));
    return PAMG_OK;
}

int face_gate_setup(pamg_handle *h) {
    if (h->gate) return PAMG_OK;
    // the stream waits on it (hipStreamWaitValue64): HIP's signal memory, as xc_sig
    HIPCHK(h, hipExtMallocWithFlags((void **)&h->gate, sizeof(unsigned long long), hipMallocSignalMemory));
    unsigned long long v = 0;
    HIPCHK(h, hipMemcpy(&v, h->gate, sizeof v, hipMemcpyDeviceToHost));
    h->gate_base = v;
    HIPCHK(h, hipHostMalloc((void **)&h->gate_stat, kGateRing * sizeof(unsigned long long), hipHostMallocCoherent));
    memset(h->gate_stat, 0, kGateRing * sizeof(unsigned long long));   // (tags start at 1)
    HIPCHK(h, hipStreamCreateWithFlags(&h->stream_fb, hipStreamNonBlocking));
    return PAMG_OK;
}

// read back the gated chain launches in stream order: each one's report arrives once it has run (its
// workgroups all resident: it opened its gate itself) or given up (the stream waits at its gate: the call
// runs here with one launch per sweep on stream_fb, from the input and snapshot the aborted launch left
// untouched, and then opens the gate). Every host wait on the handle's stream drains them first.
int face_gates_drain(pamg_handle *h) {
    if (h->agg) {   // the coarsest level's replica runs its chains on this handle's stream
        const int rc = face_gates_drain(h->agg);
        if (rc != PAMG_OK) { h->err = h->agg->err; return rc; }
    }
    while (!h->gates.empty()) {
        const pamg_handle::GatePending g = h->gates.front();
        h->gates.erase(h->gates.begin());
        volatile unsigned long long *st = h->gate_stat + (g.seq & (kGateRing - 1));
        const auto t0 = std::chrono::steady_clock::now();
        unsigned long long v = 0;
        for (unsigned i = 0;; ++i) {
            v = *st;
            if ((v >> 1) == g.seq) break;
            if ((i & 4095) != 4095) continue;
            const hipError_t e = hipStreamQuery(h->stream);
            if (e != hipSuccess && e != hipErrorNotReady) {
                h->gates.clear();
                HIPCHK(h, e);
            }
            if ((e == hipSuccess && (*st >> 1) != g.seq) ||
                std::chrono::steady_clock::now() - t0 > std::chrono::seconds(600)) {
                h->gates.clear();
                h->err = "face chain: a gated launch never reported (the state is invalid)";
                return PAMG_ERR_HIP;
            }
        }
        if (!(v & 1)) continue;
        Level &L = h->lv[g.l];
        double *const keep[3] = {L.T, L.TNN, L.RHS};
        const hipStream_t main = h->stream;
        L.T = g.T;
        L.TNN = g.TNN;
        L.RHS = g.RHS;
        h->stream = h->stream_fb;
        int rc = face_call_sweeps(h, g.l, g.sweeps, g.run, g.dead_last, g.src_is_T, g.both, false);
        if (rc == PAMG_OK && hipMemsetAsync(h->chain_tmo + 3, 0, sizeof(unsigned), h->stream) != hipSuccess) rc = PAMG_ERR_HIP;
        if (rc == PAMG_OK && hipStreamWriteValue64(h->stream, h->gate, g.want, 0) != hipSuccess) rc = PAMG_ERR_HIP;
        h->stream = main;
        L.T = keep[0];
        L.TNN = keep[1];
        L.RHS = keep[2];
        if (rc != PAMG_OK) {
            h->gates.clear();
            if (h->err.empty()) h->err = "face chain: the gated fallback failed to launch";
            return rc;
        }
        (h->tparent ? h->tparent : h)->timing.seq[PAMG_K_FACE_FALLBACK] += 1;
    }
    return PAMG_OK;
}

// res: also get_residual of level l (A tnew - RHS with the halo refreshed from tnew, :725-873) before
// the call changes tnew -- computed by the call's first tile sweep from the iterate and snapshot it
// loads anyway (the residual's own launch read tnew and RHS again), or by its own launch when the call
// runs another form
// both (not with dead_last): the call's result also into tnew -- the corrected cycle's tnew := tnew_nonlin after
// the call (smooth_to_tnew), made by the chain's final stores instead of a copy launch
int face_call(pamg_handle *h, int l, bool src_is_T, int sweeps, bool dead_last, bool res = false, bool both = false) {
    Level &L = h->lv[l];
    h->tnn_level = l;
    h->overlap_static_l1 = false;
    const double rdt = 1 / h->p.dt;
    const int kid = (l == 1) ? PAMG_K_SMOOTH_L1 : PAMG_K_SMOOTH;
    // src_is_T (the leg copy tnew_nonlin := tnew, :327 / :348 / :367): no copy launch. The call's first
    // sweep reads its iterate from tnew, which already holds what :550 would copy into it, and writes
    // tnew_nonlin for every sub-element; the halo refresh then only writes the words (it reads just the
    // sub-elements that have words). A dead-last call of one executed sweep (store 2) leaves
    // tnew_nonlin unwritten: the cycle overwrites it unread, as it does the dead sweep's.
    if (!h->tov_b) CHK(dev_alloc(h, &h->tov_b, (size_t)h->slots * 3 * std::max(h->U, 1)));
    double *buf[2] = {h->tov, h->tov_b};
    const int run = dead_last ? sweeps - 1 : sweeps;   // the sweeps that are executed
    // the residual in the first tile sweep: src_is_T (its iterate is tnew) and the tile loop below
    const bool res_in_sweep = res && src_is_T && run >= 1 && face_tile_shape(L) && !(run >= 2 && face_chain_ok(h, l)) &&
                              !face_wave_grid_for(h, l, run);
    if (res && !res_in_sweep) CHK(face_residual(h, l, false));
    if (run <= 0) {   // a call of one dead sweep: tnew := tnew_nonlin and its :555 words
        if (src_is_T && !dead_last) HIPCHK(h, launch_copy(h->stream, L.T, L.TNN, 3 * L.pitch));
        if (sweeps > 0) {
            if (src_is_T) HIPCHK(h, launch_face_words(h->stream, L, h->U, h->tov, h->tovo));
            else HIPCHK(h, launch_face_halo(h->stream, L, h->tov, h->tovo, true));
            CHK(halo(h, l));
        }
        return PAMG_OK;
    }
    if (src_is_T) HIPCHK(h, launch_face_words(h->stream, L, h->U, buf[(sweeps - 1) & 1], h->tovo));   // :555
    else HIPCHK(h, launch_face_halo(h->stream, L, buf[(sweeps - 1) & 1], h->tovo, true));   // :550, :555
    CHK(halo(h, l, buf[(sweeps - 1) & 1]));   // a partition: the remote words into the same snapshot
    // the tagged halo granules of an in-launch call (chain or wavefront): sweep s of this call carries
    // tag wave_tag + s; the base then moves past the call's tags, so no granule is ever accepted twice
    auto tags = [&](unsigned long long **g0, unsigned long long **g1, unsigned *tag0) -> int {
        CHK(face_wave_setup(h));
        const size_t ng = (size_t)h->slots * 3 * std::max(h->U, 1) * 2;
        if ((unsigned long long)h->wave_tag + sweeps + 1 >= 0xffffffffull) {   // tags would wrap: start over
            HIPCHK(h, hipMemsetAsync(h->wave_gran, 0, 2 * ng * sizeof(unsigned long long), h->stream));
            h->wave_tag = 1;
        }
        *g0 = h->wave_gran;
        *g1 = h->wave_gran + ng;
        *tag0 = h->wave_tag;
        h->wave_tag += (unsigned)sweeps + 1;
        return PAMG_OK;
    };
    unsigned long long *g0 = nullptr, *g1 = nullptr;
    unsigned tag0 = 0;
    if (run >= 2 && face_chain_ok(h, l)) {   // the whole call in one launch
        CHK(face_chain_setup(h, l));
        if ((unsigned long long)L.chain_epoch + run + 2 >= 0xffffffffull) {   // the epoch would wrap: start over
            HIPCHK(h, hipMemsetAsync(L.chain_flags, 0, L.chain_flag_bytes, h->stream));
            L.chain_epoch = 0;
        }
        const unsigned f0 = L.chain_epoch;
        L.chain_epoch += (unsigned)run + 1;
        ChainGate G;
        CHK(face_gate_setup(h));
        if (h->gates.size() >= kGateRing / 2) CHK(face_gates_drain(h));   // (the status ring's reuse)
        G.gate = h->gate;
        G.stat = h->gate_stat;
        G.seq = h->gate_seq;
        {
            // the state crosses HBM once per call: tnew_nonlin and RHS in, tnew (+ tnew_nonlin) out
            Span sp(h, kid, (dead_last ? 72.0 : 96.0) * (double)L.N + 168.0 * h->U);
            h->chain_pending = true;
            HIPCHK(h, launch_face_chain(h->stream, L, h->U, h->cus, h->tov, h->tov_b, h->tovo, L.chain_flags,
                                        L.chain_nb_off, L.chain_nb_list, h->chain_tmo, run, sweeps,
                                        dead_last ? 2 : both ? 3 : 1,
                                        h->p.solver == 3, l == 1, rdt, h->p.omega, h->slots, src_is_T, f0, 1, G));
        }
        // fail safe: a launch whose workgroups were not all resident (a CU-masked stream, another stream's or
        // process's kernels on the CUs) aborted before touching anything -- the call runs with one launch per
        // sweep, from the same input and halo snapshot: the stream waits for the launch's report at its gate and
        // the host runs the fallback when it reads the report back (face_gates_drain, at the latest when the API
        // call ends). (Round 5's first form, the host waiting for every launch, cost 2.3 % more; removed.)
        h->gate_seq += 1;
        h->gate_base += 1;
        HIPCHK(h, hipStreamWaitValue64(h->stream, h->gate, h->gate_base, hipStreamWaitValueGte));
        h->gates.push_back({G.seq, h->gate_base, l, sweeps, run, dead_last, src_is_T, both, L.T, L.TNN, L.RHS});
        return PAMG_OK;
    }
    if (const int g = face_wave_grid_for(h, l, run)) {   // the call in one wavefront launch
        CHK(tags(&g0, &g1, &tag0));
        // the state crosses HBM once per call, as the chain's
        Span sp(h, kid, (dead_last ? 72.0 : 96.0) * (double)L.N + 168.0 * h->U);
        h->chain_pending = true;
        HIPCHK(h, launch_face_wave(h->stream, L, h->U, g, h->tov, h->tov_b, h->tovo, g0, g1, tag0, h->wave_flags,
                                   h->wave_order, h->chain_tmo, run, sweeps, dead_last ? 2 : 1, h->p.solver == 3,
                                   l == 1, rdt, h->slots, src_is_T));
        if (both) HIPCHK(h, launch_copy(h->stream, L.TNN, L.T, 3 * L.pitch));
        return PAMG_OK;
    }
    return face_call_sweeps(h, l, sweeps, run, dead_last, src_is_T, both, res_in_sweep);
}

// `sweeps` sweeps on level l reading the iterate from T (src_is_T: the leg
// copy tnew_nonlin := tnew is folded into the launch) or from TNN.
int smooth(pamg_handle *h, int l, bool src_is_T, int sweeps) {
    Level &L = h->lv[l];
    h->tnn_level = l;
    h->overlap_static_l1 = false;   // the per-step smoother writes every halo word of level l
    if (sweeps <= 0) {
        if (src_is_T) HIPCHK(h, launch_copy(h->stream, L.T, L.TNN, 3 * L.pitch));
        return PAMG_OK;
    }
    const double rdt = 1 / h->p.dt;
    const int kid = (l == 1) ? PAMG_K_SMOOTH_L1 : PAMG_K_SMOOTH;
    const double bytes = 96.0 * (double)L.N + 168.0 * h->U;
    if (h->p.op == 1) {   // face-coupled operator: the halo is read, so it is refreshed (and exchanged) every sweep
        // single domain: one launch per sweep (PAMG_FACE_FUSED=0: the per-colour sequence)
        if (face_fusable(h, l)) return face_call(h, l, src_is_T, sweeps, false);
        if (src_is_T) HIPCHK(h, launch_copy(h->stream, L.T, L.TNN, 3 * L.pitch));
        // a partition: per sweep the halo refresh, the exchange, then the sweep itself -- one tile
        // launch (both colours on the iterate in LDS, reading the exchanged t_overlap) or the two
        // colour kernels
        const bool tiles = face_tiles_ok(h, l);
        for (int s = 0; s < sweeps; ++s) {
            HIPCHK(h, launch_face_halo(h->stream, L, h->tov, h->tovo, true));   // tnew := tnew_nonlin (:550), :555
            CHK(halo(h, l));
            Span sp(h, kid, tiles ? 72.0 * (double)L.N + 168.0 * h->U : bytes + 72.0 * (double)L.N);
            if (tiles) {   // tnew_nonlin only: the refresh has copied tnew := tnew_nonlin
                HIPCHK(h, launch_face_sweep_fused(h->stream, L, h->tov, nullptr, h->tovo, h->p.solver == 3, l == 1, rdt,
                                                  h->p.omega, h->slots, 0, false));
            } else if (h->p.solver == 3) {   // red-black Gauss-Seidel: up sub-elements, then down ones
                HIPCHK(h, launch_face_sweep(h->stream, L, h->tov, 0, l == 1, rdt, h->p.omega, h->slots));
                HIPCHK(h, launch_face_sweep(h->stream, L, h->tov, 1, l == 1, rdt, h->p.omega, h->slots));
            } else {
                HIPCHK(h, launch_face_sweep(h->stream, L, h->tov, 2, l == 1, rdt, h->p.omega, h->slots));
            }
        }
        return PAMG_OK;
    }
    if (h->p.halo_mode == 1) {
        for (int s = 0; s < sweeps; ++s) {
            {
                Span sp(h, kid, bytes);
                HIPCHK(h, launch_smooth(h->stream, L, (s == 0 && src_is_T) ? L.T : L.TNN, 1, h->p.solver, rdt,
                                        h->p.omega, h->tov, h->tovo));
            }
            CHK(halo(h, l));
        }
        return PAMG_OK;
    }
    {
        Span sp(h, kid, bytes);
        HIPCHK(h, launch_smooth(h->stream, L, src_is_T ? L.T : L.TNN, sweeps, h->p.solver, rdt, h->p.omega, h->tov,
                                h->tovo));
    }
    return halo(h, l);
}

// PAMG_RHS_TOLD_HALO (A/B builds): k_rhs writes the compact told copy of the halo at the start of a
// step (1) or k_told_halo gathers it afterwards (0, default: the folded form measured 1.4 % slower
// on the time loop, scripts/ab_tl.sh, profiles/r01_v17_time_loop.txt)
#ifndef PAMG_RHS_TOLD_HALO
#define PAMG_RHS_TOLD_HALO 0
#endif
int rhs_level1(pamg_handle *h, int start_of_step) {
    Level &L = h->lv[1];
    Span sp(h, PAMG_K_RHS, (start_of_step == 1 ? 96.0 : start_of_step == 2 ? 72.0 : 48.0) * (double)L.N);
    HIPCHK(h, launch_rhs(h->stream, L, 1 / h->p.dt, start_of_step, PAMG_RHS_TOLD_HALO && start_of_step != 0));
    return PAMG_OK;
}

int residual(pamg_handle *h, int l);
int restrict_(pamg_handle *h, int l);

// told changed on level l: refresh the compact told copy the halo reads
int refresh_told_halo(pamg_handle *h, int l) {
    h->overlap_static_l1 = false;
    if (l == 1) h->told_halo_stale_l1 = false;
    HIPCHK(h, launch_told_halo(h->stream, h->lv[l], h->U));
    return PAMG_OK;
}

// restrictor(l) + get_residual(l) as one kernel (V-cycle driver)
int restrict_residual(pamg_handle *h, int l) {
    Level &L = h->lv[l];
    h->rhsn_valid = false;
    if (l >= h->p.multi_levels || h->p.op == 1) {
        CHK(restrict_(h, l));
        return residual(h, l);
    }
    if (l == 1 && h->p.solver == 2) CHK(rhs_level1(h, 0));   // get_RHS inside get_residual (:865-867)
    Span sp(h, PAMG_K_RESIDUAL, 102.0 * (double)L.N + 168.0 * h->U);
    HIPCHK(h, launch_restrict_residual(h->stream, L, h->lv[l + 1], 1 / h->p.dt));
    return PAMG_OK;
}

// face-coupled operator: residual A tnew - RHS (neg: RHS - A tnew) with the halo refreshed from tnew
int face_residual(pamg_handle *h, int l, bool neg) {
    Level &L = h->lv[l];
    h->rhsn_valid = false;
    h->overlap_static_l1 = false;
    HIPCHK(h, launch_face_words(h->stream, L, h->U, h->tov, h->tovo));
    CHK(halo(h, l));
    // tnew, RHS in, residual out (the neighbours' values are the same tnew, gathered from cache)
    Span sp(h, PAMG_K_RESIDUAL, 72.0 * (double)L.N + 168.0 * h->U);
    HIPCHK(h, launch_face_residual(h->stream, L, h->tov, neg, l == 1, 1 / h->p.dt, h->slots));
    return PAMG_OK;
}

int residual(pamg_handle *h, int l) {
    Level &L = h->lv[l];
    if (h->p.op == 1) return face_residual(h, l, false);
    h->rhsn_valid = false;
    if (l == 1 && h->p.solver == 2) CHK(rhs_level1(h, 0));   // get_RHS inside get_residual (:865-867)
    Span sp(h, PAMG_K_RESIDUAL, 72.0 * (double)L.N + 168.0 * h->U);
    HIPCHK(h, launch_residual(h->stream, L, 1 / h->p.dt));
    return PAMG_OK;
}

int restrict_(pamg_handle *h, int l) {
    if (l >= h->p.multi_levels) return PAMG_OK;   // splitting.F90:18
    Span sp(h, PAMG_K_RESTRICT, 96.0 * (double)h->lv[l + 1].N);
    HIPCHK(h, launch_restrict(h->stream, h->lv[l], h->lv[l + 1], h->U));
    return PAMG_OK;
}

int prolong(pamg_handle *h, int l, bool fused_copy) {
    if (l >= h->p.multi_levels) { h->err = "prolongator needs a coarser level"; return PAMG_ERR_ARG; }
    if (fused_copy) h->tnn_level = l;
    Span sp(h, PAMG_K_PROLONG, (fused_copy ? 312.0 : 216.0) * (double)h->lv[l + 1].N);
    HIPCHK(h, launch_prolong(h->stream, h->lv[l], h->lv[l + 1], fused_copy));
    return PAMG_OK;
}

// algorithmic HBM bytes of the two fused V-cycle launches: the state each
// launch must read and write once, plus the operator words it reads (c, Kd, omega/D: 104 B
// per un_ele and level)
//   level-1 launch: level 1 reads tnew, RHS and writes residual, tnew, tnew_nonlin (120 B);
//                   level 2 reads the final tnew (prolongator) and writes RHSN (48 B)
//   coarse launch:  level l >= 2 reads tnew, RHSN and writes RHS, residual, tnew (120 B);
//                   RHSN of the levels l >= 3 is written here too (24 B)
double vcycle_fine_bytes(pamg_handle *h, int keep = PAMG_KEEP_ALL) {
    const int L = h->p.multi_levels;
    return (keep & PAMG_KEEP_L1 ? 120.0 : 72.0) * h->lv[1].N + (L > 1 ? 48.0 * h->lv[2].N : 0.0) + 104.0 * h->U;
}
double vcycle_coarse_bytes(pamg_handle *h, int keep = PAMG_KEEP_ALL) {
    const int L = h->p.multi_levels;
    double b = 0.0;
    for (int l = 2; l <= L; ++l) b += (120.0 - (keep & PAMG_KEEP_COARSE ? 0.0 : 48.0) + (l >= 3 ? 24.0 : 0.0)) * h->lv[l].N;
    return b + 104.0 * h->U * (L - 1);
}
//   pipelined launch: both, less level 2's RHSN (written and read: 48 B) and its tnew read
//                     by the coarse part (the level-1 part's read serves both: 24 B), less
//                     the dead-until-final stores it skips (keep, PAMG_KEEP_*): level 1's
//                     residual and tnew_nonlin (48 B), the coarse levels' RHS and residual
//                     (48 B); the halo words are not counted anywhere
double vcycle_pipe_bytes(pamg_handle *h, int keep) {
    double b = vcycle_fine_bytes(h) + vcycle_coarse_bytes(h) - 72.0 * h->lv[2].N;
    if (!(keep & PAMG_KEEP_L1)) b -= 48.0 * h->lv[1].N;
    if (!(keep & PAMG_KEEP_COARSE))
        for (int l = 2; l <= h->p.multi_levels; ++l) b -= 48.0 * h->lv[l].N;
    return b;
}
//   resident launch (a whole call): every level's state in and out once -- level 1 reads
//                     tnew and RHS (the source s' when it starts a step) and writes tnew,
//                     and with PAMG_KEEP_L1 its residual and tnew_nonlin (and the RHS it
//                     formed); told with PAMG_KEEP_TOLD; a coarse level reads tnew and RHSN
//                     and writes tnew and RHSN (level 2's RHSN: the restriction of level 1's
//                     last residual), with PAMG_KEEP_COARSE its RHS and residual
double vcycle_res_bytes(pamg_handle *h, int keep, bool rhsf) {
    const int L = h->p.multi_levels;
    double b = (72.0 + (keep & PAMG_KEEP_L1 ? (rhsf ? 72.0 : 48.0) : 0.0) + (keep & PAMG_KEEP_TOLD ? 24.0 : 0.0)) *
               h->lv[1].N;
    for (int l = 2; l <= L; ++l) b += (96.0 + (keep & PAMG_KEEP_COARSE ? 48.0 : 0.0)) * h->lv[l].N;
    return b + 104.0 * h->U * L;
}
// fp64 operations one V-cycle of the fused forms executes (fma = 2): a sweep is 12 fma (24 flop,
// contracted) or 42 operations (the reference's order, apply_A + update), get_residual 9 fma or
// 36; the restrictor's input mean 3 per sub-element of the levels < L; the prolongator cascade 21
// per coarse sub-element (splitting.F90:59-88, executed on LDS images although its output is dead).
// A smoother call's last sweep only produces tnew_nonlin; inside a fused cycle that value is
// overwritten before any read (:367 after the restriction leg, :327 of the next cycle after the
// prolongation leg, :348 on the coarsest level), so it is never computed (the compiler drops it:
// its result never leaves registers) -- per cycle a level l < L runs 2 (n_smooth - 1) sweeps and
// the coarsest n_smooth (1 + n_coarse) - 2; only a call's last cycle also runs level 1's final
// sweep, whose tnew_nonlin it stores (not counted here)
int call_schedule(pamg_handle *h);
bool corrected_resident_ok(pamg_handle *h);
double vcycle_flops(pamg_handle *h) {
    const int L = h->p.multi_levels, ns = h->p.n_smooth, nc = h->p.n_coarse;
    const bool f = h->p.arith == 1 && h->p.solver != 2;
    // Richardson's update is x + omega b (a multiply and an add per component), its residual the
    // reference's order
    const double sw = h->p.solver == 2 ? 6.0 : f ? 24.0 : 42.0, rs = f ? 18.0 : 36.0;
    if (h->p.cycle == 1) {
        // the corrected cycle: every sweep is live -- a level l < L runs two calls of n_smooth sweeps, the
        // fresh residual and its mean (3), and takes the interpolated correction (3 adds per sub-element,
        // the three midpoints, 9 flops, per coarse parent); the coarsest n_coarse calls from zero; the fine
        // residual after the cycle only in a call's last cycle (not counted)
        double fl = 0.0;
        for (int l = 1; l <= L; ++l) {
            const double n = (double)h->lv[l].N;
            if (l < L) fl += n * (2.0 * ns * sw + rs + 3.0 + 3.0) + 9.0 * (double)h->lv[l + 1].N;
            else fl += n * ((double)ns * (L > 1 ? nc : 1) * sw + (L > 1 ? 0.0 : rs));
        }
        return fl;
    }
    // the resident kernels (call schedule 3) do not compute the dead prolongator (pamg_vcycle.hip
    // k_vc_res, k_vc_resb); every other fused form executes its cascade
    const bool prolong = !(call_schedule(h) == 3 && vcycle_resident_supported(h->p.n_split, L));
    double fl = 0.0;
    for (int l = 1; l <= L; ++l) {
        const double n = (double)h->lv[l].N;
        if (l < L) fl += n * (2.0 * std::max(ns - 1, 0) * sw + rs + 3.0);
        else fl += n * ((nc > 0 ? (double)ns * (1 + nc) - 2 : (double)ns - 1) * sw + rs);
        if (l >= 2 && prolong) fl += n * 21.0;
    }
    return fl;
}
// the stores a pipelined launch makes beyond what the call needs: none (forcing them, the round-2 A/B, moved
// 120 instead of 72 B per level-1 sub-element)
constexpr int kPipeKeep = 0;

// the exact local solve of level l (coarse_solver = 1): tnew = tnew_nonlin = A_e^-1 RHS, with
// A_e^-1 from FINDInv, formed on first use
int direct_solve(pamg_handle *h, int l) {
    Level &L = h->lv[l];
    if (!L.Ainv) {
        int *d_err = nullptr;
        CHK(dev_alloc(h, &L.Ainv, 9 * (size_t)std::max(h->U, 1)));
        HIPCHK(h, hipMalloc((void **)&d_err, sizeof(int) * std::max(h->U, 1)));
        HIPCHK(h, launch_block_ops(h->stream, L, h->U, 1 / h->p.dt, L.Ainv, d_err));
        std::vector<int> err(std::max(h->U, 1));
        HIPCHK(h, hipMemcpyAsync(err.data(), d_err, sizeof(int) * h->U, hipMemcpyDeviceToHost, h->stream));
        CHK(sync_stream(h, h->stream));   // (the gates first: hipFree waits for the whole device)
        (void)hipFree(d_err);
        for (int q = 0; q < h->U; ++q)
            if (err[q]) {
                h->err = "FINDInv: operator block of un_ele " + std::to_string(h->owned[q] + 1) + " on level " +
                         std::to_string(l) + " is not invertible";
                return PAMG_ERR_STATE;
            }
    }
    h->tnn_level = l;
    HIPCHK(h, launch_block_solve(h->stream, L, L.Ainv));
    return PAMG_OK;
}

// one V-cycle as the per-step kernel sequence of transport_tri_semi.F90:319-379
int vcycle_steps(pamg_handle *h) {
    const int L = h->p.multi_levels, ns = h->p.n_smooth;
    for (int l = 1; l <= L; ++l) {           // :323-340
        CHK(smooth(h, l, true, ns));
        CHK(restrict_residual(h, l));
    }
    if (h->p.coarse_solver == 1) CHK(direct_solve(h, L));   // the direct path instead of :344-359
    else CHK(smooth(h, L, true, ns * h->p.n_coarse));   // :344-359
    for (int l = L - 1; l >= 1; --l) {             // :363-378
        CHK(prolong(h, l, true));
        CHK(smooth(h, l, false, ns));
    }
    return PAMG_OK;
}

// The face-coupled operator's V-cycle (op = 1, cycle = 0) on a single domain, as the per-step
// sequence above with its dead work dropped: a smoother call's last sweep only makes a
// tnew_nonlin that the cycle overwrites before any read (:367 after the restriction leg, :348 at the
// coarsest level, the next cycle's :327 after the prolongation leg), so it runs only in the call's
// last cycle, where it is observable; the sweep before it leaves tnew and the dead sweep's halo words
// (face_call), which are also what get_residual's refresh from tnew (:555 via update_overlaps) would
// write, so the residual reads them as they are; the prolongator's output is overwritten by the
// smoother's first statement (:550, SURVEY.md A3 iv) and is not computed. The state after a call --
// every field of every level, t_overlap, t_overlap_old -- is bitwise the per-step sequence's
// (tests/test_face_operator.py).
bool face_cycle_fusable(pamg_handle *h) {
    if (!(h->p.fused && h->p.op == 1 && h->p.cycle == 0 && h->p.coarse_solver == 0)) return false;
    for (int l = 1; l <= h->p.multi_levels; ++l)
        if (!face_fusable(h, l)) return false;
    return true;
}

// ---- the face V-cycle with two sweeps per HBM pass (k_face_pp) on the levels below the coarsest
// The fused cycle's level-l work, for l < L, is a stream of sweeps on one RHS: its restriction-leg call's
// executed sweeps and its prolongation-leg call's, which starts from the restriction-leg tnew (:367; the
// prolongated values are overwritten unread, :550), with get_residual between them -- and level 1's RHS
// is the time step's, so level 1's streams of all the call's cycles are ONE stream (its coarse levels
// never feed back into it). Such a stream runs as launches of two sweeps (the halo of the second sweep
// computed in the launch, k_face_pp), the residual inside the launch that passes its point, and the
// state rotating through tnew, tnew_nonlin and RHSN (op = 1 has no use for RHSN) -- a launch never writes
// the iterate its neighbours read. The restrictor of level l (:336, the PREVIOUS residual) runs before the
// launch that writes the new one; a coarse level's whole cycle runs before the next level's (nothing of
// the next level reaches it). The halo words (:555) are no longer published between sweeps (the launches
// read the iterate itself): t_overlap, t_overlap_old and the boundary words are written from level 1's
// tnew once, after the call -- what the per-step sequence's last writer, level 1's last smoother call,
// leaves (every coarser level writes a subset of its slots). Bitwise the per-step sequence
// (tests/test_face_operator.py). PAMG_FACE_PP=0 keeps the one-sweep launches (A/B).
// PAMG_FACE_PP: a mask of the level sizes that stream -- bit 0 levels of 1,024 sub-elements per un_ele,
// bit 1 of 256; 0 none. Default 3: both (the 256-element passes were slower while their instance
// spilled at six waves per SIMD, profiles/r04_d_face_pp.txt; at four, 620 vs 601-603 V-cycles/s with
// level 1 alone, profiles/r04_i_face_pp_level2.txt)
bool face_pp_ok(pamg_handle *h, int l) {
    const char *ev = getenv("PAMG_FACE_PP");   // read per call: tests switch it within a process
    const int mask = ev ? atoi(ev) : 3;
    const Level &L = h->lv[l];
    const int bit = L.nsub == 1024 ? 1 : L.nsub == 256 ? 2 : 0;
    // a single domain: the passes read the neighbours' iterate itself
    return (mask & bit) && face_fusable(h, l) && h->nranks == 1 && !h->comm && face_tile_shape(L) && L.gtab &&
           (h->p.solver != 3 || L.words_up);
}

// a pass of a face stream (face_pp_plan); rhsc: its residual also restricted into this buffer (res_drop: and not
// stored), interp: the coarse correction added to its loads (PPCoarse)
struct PPPass {
    int K, res;
    double *in, *pre, *mid, *end, *end2;
    bool interp = false;
    double *rhsc = nullptr;
    bool res_drop = false;
};

// the passes of a stream of `total` sweeps from src with get_residual after sweep r for each r in res_at
// (0 < r < total), ending with the final stores fin (1: tnew = the iterate before the last sweep,
// tnew_nonlin = after it; 2: tnew = the last result, the dead sweep's :550; 3: tnew and tnew_nonlin both
// the last result, the corrected cycle's smoother call)
int face_pp_plan(pamg_handle *h, int l, int total, double *src, const std::vector<int> &res_at, int fin,
                 std::vector<PPPass> &plan) {
    Level &L = h->lv[l];
    plan.clear();
    for (int s = 0; s < total; s += 2)
        plan.push_back(PPPass{std::min(2, total - s), 0, nullptr, nullptr, nullptr, nullptr, nullptr});
    for (int r : res_at) {
        if (r <= 0 || r >= total) { h->err = "internal: face stream residual point"; return PAMG_ERR_STATE; }
        PPPass &q = plan[r / 2];
        if (q.res) { h->err = "internal: two residuals in one face pass"; return PAMG_ERR_STATE; }
        q.res = (r & 1) ? 2 : 1;   // after the pass's first sweep, or at its start
    }
    const int P = (int)plan.size();
    PPPass &z = plan[P - 1];
    if (fin == 1) {
        if (z.K == 2) z.mid = L.T; else z.pre = L.T;
        z.end = L.TNN;
    } else {
        z.end = L.T;
        if (fin == 3) z.end2 = L.TNN;
    }
    double *const buf[3] = {L.RHSN, L.TNN, L.T};
    // inputs, last to first: the last pass reads RHSN (neither of its outputs); every other pass writes the
    // next one's input, which is not its own; the first reads src
    std::vector<double *> in(P);
    in[P - 1] = P == 1 ? src : L.RHSN;
    for (int p = P - 2; p >= 1; --p)
        for (double *b : buf)
            if (b != in[p + 1] && (p != 1 || b != src)) { in[p] = b; break; }
    if (P >= 2) in[0] = src;
    for (int p = 0; p < P; ++p) {
        plan[p].in = in[p];
        if (p + 1 < P) plan[p].end = in[p + 1];
        if (plan[p].in && (plan[p].in == plan[p].end || plan[p].in == plan[p].mid || plan[p].in == plan[p].pre ||
                           plan[p].in == plan[p].end2)) {   // (in null: a start from zero reads nothing)
            h->err = "internal: a face pass writes its own input";
            return PAMG_ERR_STATE;
        }
    }
    return PAMG_OK;
}

int face_pp_emit(pamg_handle *h, int l, const PPPass &q) {
    Level &L = h->lv[l];
    const int kid = (l == 1) ? PAMG_K_SMOOTH_L1 : PAMG_K_SMOOTH;
    // iterate and RHS in, the outputs and the residual out (the halo gathers of the neighbours' boundary
    // sub-elements are overhead, not counted)
    // (a start from zero reads no iterate; the folded interpolation reads the coarse level's, 6 B per sub-element)
    const double by = (24.0 * (q.in != nullptr) + 24.0 + (q.interp ? 6.0 : 0.0) + (q.rhsc ? 6.0 : 0.0) +
                       24.0 * ((q.pre != nullptr) + (q.mid != nullptr) + (q.end != nullptr) + (q.end2 != nullptr) +
                               (q.res != 0 && !q.res_drop))) * (double)L.N + 168.0 * h->U;
    if (q.res) h->rhsn_valid = false;
    Span sp(h, kid, by);
    PPCoarse pc;
    pc.coarse = (q.interp || q.rhsc) ? &h->lv[l + 1] : nullptr;
    pc.rhsc = q.rhsc;
    pc.res_store = !q.res_drop;
    pc.interp = q.interp;
    HIPCHK(h, launch_face_pp(h->stream, L, q.K, q.in, q.pre, q.mid, q.end, h->p.solver == 3, l == 1, 1 / h->p.dt, q.res,
                             q.end2, pc.coarse ? &pc : nullptr));
    return PAMG_OK;
}

// the coarsest level's two smoother calls of a cycle that is not the call's last as ONE call: the restriction
// leg's (:331, ns sweeps, the last dead: tnew := sweep ns - 1) and the coarse solve's (:344-359, ns n_coarse
// sweeps from tnew, the last dead). Between them the cycle computes only the coarsest residual (:338), which
// such a cycle skips (face_pp_level), and the second call's leg copy tnew_nonlin := tnew (:348) continues from
// the first call's tnew: one call of (ns - 1) + (ns n_coarse - 1) executed sweeps and a dead last one, whose
// halo words at the seam are the ones the first call's last executed sweep published -- the words of that tnew,
// as the second call's refresh would write them. (The two calls run in a call's last cycle, whose residual is
// state; the merged form is bitwise them: tests/test_face_operator.py, oracle parity.)
bool face_coarse_merged(pamg_handle *h, bool last) {
    return !last && h->p.n_smooth >= 1 && h->p.n_coarse >= 1;
}

// :336 for level l >= 2 of the face cycle: the restriction of level l's previous residual into level l+1's RHS -- the
// buffer a fold made in the previous cycle's pass (swapped in), else the restrictor
int face_restrict_prev(pamg_handle *h, int l) {
    if (h->pp_folded[l]) {
        std::swap(h->lv[l + 1].RHS, h->lv[l + 1].RHSN_alt);
        h->pp_folded[l] = false;
        return PAMG_OK;
    }
    return restrict_(h, l);
}

// level l's part of cycle c of the fused face cycle (levels l .. L): the coarsest level's calls; a level
// below it as a two-sweep stream (its restrictor before the launch that writes its new residual, then the
// next level), or as its two calls around the next level (vcycle_face_fused's order)
int face_pp_level(pamg_handle *h, int l, bool last) {
    const int L = h->p.multi_levels, ns = h->p.n_smooth;
    const double rdt = 1 / h->p.dt;
    if (l == L) {
        if (face_coarse_merged(h, last)) return face_call(h, L, true, ns + ns * h->p.n_coarse - 1, true);
        CHK(face_call(h, l, true, ns, true));   // :331 via :351
        Level &V = h->lv[l];
        h->rhsn_valid = false;
        // the coarsest level's get_residual (:338): nothing restricts or reads it (restrictor(L) is empty,
        // splitting.F90:18), and the next cycle rewrites it -- only the call's last cycle's is state
        if (last) {
            Span sp(h, PAMG_K_RESIDUAL, 72.0 * (double)V.N + 168.0 * h->U);
            HIPCHK(h, launch_face_residual(h->stream, V, h->tov, false, l == 1, rdt, h->slots));
        }
        return face_call(h, L, true, ns * h->p.n_coarse, !last);   // :344-359
    }
    if (!face_pp_ok(h, l) || 2 * (ns - 1) + (last ? 1 : 0) < 3) {   // (one pass could not rotate its buffers)
        CHK(face_call(h, l, true, ns, true));
        CHK(face_restrict_prev(h, l));
        CHK(face_pp_level(h, l + 1, last));
        return face_call(h, l, true, ns, !last, true);
    }
    h->tnn_level = l;
    h->overlap_static_l1 = false;
    std::vector<PPPass> plan;
    CHK(face_pp_plan(h, l, 2 * (ns - 1) + (last ? 1 : 0), h->lv[l].T, {ns - 1}, last ? 1 : 2, plan));
    // the restrictor folded (vcycle_face_pp's level-1 fold, one level down): the pass that computes this cycle's
    // residual restricts it into level l+1's RHSN_alt and, but in the call's last cycle, does not store it (only
    // the restrictor reads it); the next cycle swaps that buffer in where it would restrict
    const bool fold = h->pp_fold && h->lv[l + 1].RHSN_alt;
    bool restricted = false;
    for (const PPPass &q : plan) {
        if (q.res && !restricted) { CHK(face_restrict_prev(h, l)); restricted = true; }   // :336, the previous residual
        PPPass qf = q;
        if (q.res && fold && !last) {
            qf.rhsc = h->lv[l + 1].RHSN_alt;
            qf.res_drop = true;
        }
        CHK(face_pp_emit(h, l, qf));
        if (qf.rhsc) h->pp_folded[l] = true;
    }
    if (!restricted) CHK(face_restrict_prev(h, l));
    return face_pp_level(h, l + 1, last);
}

int vcycle_face_pp(pamg_handle *h, int n) {
    const int ns = h->p.n_smooth;
    if (n <= 0) return PAMG_OK;
    if (!face_pp_ok(h, 1)) {   // level 1 as its two calls per cycle, a coarser level as a stream
        for (int c = 0; c < n; ++c) CHK(face_pp_level(h, 1, c + 1 == n));
        h->tnn_level = 1;
        return face_chain_check(h);
    }
    // level 1: one stream over the call's cycles, get_residual after each cycle's restriction leg
    const int per = 2 * (ns - 1);
    std::vector<int> res_at;
    for (int c = 0; c < n; ++c) res_at.push_back(ns - 1 + per * c);
    std::vector<PPPass> plan;
    CHK(face_pp_plan(h, 1, per * n + 1, h->lv[1].T, res_at, 1, plan));
    h->overlap_static_l1 = false;
    // the restrictor folded into the pass that computes the residual (PAMG_FACE_RR=0: its own launch). The cycle
    // restricts the PREVIOUS cycle's residual (:336 before :338), so the pass that computes cycle c's residual
    // restricts it into level 2's second RHS buffer (RHSN_alt, unused by the face cycle) and cycle c + 1 swaps the
    // two instead of launching the restrictor; that residual is then not stored either (only the restrictor reads
    // it) -- except the call's last cycle's, which is the state, and which the next call's first cycle restricts
    const char *rr_env = getenv("PAMG_FACE_RR");
    Level &L2 = h->lv[2];
    const bool rf = !(rr_env && atoi(rr_env) == 0) && h->p.multi_levels >= 2 && L2.RHSN_alt;
    // levels 2 .. L: each RHS's own buffer (the folds swap RHS and RHSN_alt). An error return inside the loop leaves
    // the buffers as it found them (the state is invalid after an error, but RHS and RHSN_alt stay the handle's own
    // two buffers in their roles); the coarse levels' folds are off outside this call
    const int Lc = h->p.multi_levels;
    double *rhs_home[kMaxLevels + 1] = {};
    for (int l = 2; l <= Lc; ++l) rhs_home[l] = h->lv[l].RHS;
    struct Home {
        pamg_handle *h; int Lc; double *const *home;
        ~Home() {
            for (int l = 2; l <= Lc; ++l)
                if (h->lv[l].RHS != home[l]) std::swap(h->lv[l].RHS, h->lv[l].RHSN_alt);
            h->pp_fold = false;
            for (bool &f : h->pp_folded) f = false;
        }
    } home_guard{h, Lc, rhs_home};
    h->pp_fold = rf;
    size_t p = 0;
    for (int c = 0; c < n; ++c) {
        h->tnn_level = 1;
        if (c == 0 || !rf) CHK(restrict_(h, 1));   // :336 -- level 1's residual of the previous cycle, before this cycle's is written
        else std::swap(L2.RHS, L2.RHSN_alt);       // the restriction of it, made by the pass that computed it
        const size_t pr = (size_t)res_at[c] / 2;   // the pass that writes this cycle's residual
        for (; p <= pr; ++p) {
            PPPass q = plan[p];
            if (p == pr && rf && c + 1 < n) {
                q.rhsc = L2.RHSN_alt;
                q.res_drop = true;
            }
            CHK(face_pp_emit(h, 1, q));
        }
        CHK(face_pp_level(h, 2, c + 1 == n));
    }
    for (; p < plan.size(); ++p) CHK(face_pp_emit(h, 1, plan[p]));
    for (int l = 2; l <= Lc; ++l) {   // each RHS back in its own buffer
        Level &V = h->lv[l];
        if (V.RHS == rhs_home[l]) continue;
        HIPCHK(h, hipMemcpyAsync(V.RHSN_alt, V.RHS, 3 * (size_t)V.pitch * sizeof(double), hipMemcpyDeviceToDevice, h->stream));
        std::swap(V.RHS, V.RHSN_alt);
    }
    // the halo the per-step sequence leaves: level 1's last smoother call's words, from its tnew (:555)
    HIPCHK(h, launch_face_words(h->stream, h->lv[1], h->U, h->tov, h->tovo));
    h->tnn_level = 1;
    return face_chain_check(h);
}

// ---- op = 1 on a partition: the coarsest level agglomerated ----------------------------
// On a partition the coarsest level's smoother calls -- 62 of the cycle's 74 sweeps at the bench shape, each
// reading the halo words the neighbours' previous sweep wrote -- would be one launch and one exchange per sweep.
// The level is small (12.6 MB per field for all of untitled8192 at n_split 5) and, in the reference's cycle,
// nothing finer reads it back within a call (the prolongator's output is overwritten, SURVEY.md A3 iv); in the
// corrected cycle only its result is read. So every rank gathers the ranks' blocks of the level's RHS (the
// restriction of their own level-2 residuals, splitting.F90:10-32) into a replica of the WHOLE level (h->agg,
// single domain, renumbered rank block by rank block) and runs there the single-domain coarsest calls
// (transport_tri_semi.F90:331 via :351, :338, :344-359): the persistent chain, its halo words handed over inside
// the launch. The replicas stay identical on every rank (the same inputs through the same kernels), and a rank
// copies its own block of the result back into its level L. The replica's tnew carries over from call to call as
// the level's tnew does (it is never reset, A3 v); it is gathered from the ranks once at the start of each call,
// so a partition's level L written between calls by anything else (pamg_set_state, per-step calls) is picked up.
// Bitwise the single domain (tests/test_face_operator.py). PAMG_FACE_AGG=0 at upload keeps the per-sweep form.

// the local-group transport: every peer's block of a 3-plane field pulled from its handle, behind its event
int gather_local(pamg_handle *h, const double *local, int64_t lpitch, double *rep, int64_t rpitch, int nsub,
                 hipStream_t st) {
    Comm &C = *h->comm;
    LocalGroup &G = *C.local;
    const int me = h->rank, n = G.n;
    std::vector<LocalGroup::Post> got(n);
    auto wait_posts = [&](std::vector<LocalGroup::Post> &box, const char *what) -> int {
        std::unique_lock<std::mutex> lk(G.mu);
        for (int peer = 0; peer < n; ++peer) {
            if (peer == me) continue;
            const long want = C.seq[peer] + 1;
            LocalGroup::Post &b = box[(size_t)peer * n + me];
            if (!G.cv.wait_for(lk, std::chrono::seconds(local_timeout_s()), [&] { return b.seq >= want; })) {
                h->err = "local coarse gather: rank " + std::to_string(me) + " timed out waiting for rank " +
                         std::to_string(peer) + "'s " + what;
                return PAMG_ERR_COMM;
            }
            if (b.seq != want) { h->err = "local coarse gather: sequence mismatch"; return PAMG_ERR_COMM; }
            got[peer] = b;
        }
        return PAMG_OK;
    };
    HIPCHK(h, hipEventRecord(C.ev_ready, st));
    {
        std::lock_guard<std::mutex> lk(G.mu);
        for (int peer = 0; peer < n; ++peer)
            if (peer != me) G.ready[(size_t)me * n + peer] = {C.seq[peer] + 1, local, C.ev_ready, lpitch};
    }
    G.cv.notify_all();
    CHK(wait_posts(G.ready, "coarse block"));
    for (int peer = 0; peer < n; ++peer) {
        if (peer == me) continue;
        const size_t cnt = (size_t)(h->agg_off[peer + 1] - h->agg_off[peer]) * nsub;
        HIPCHK(h, hipStreamWaitEvent(st, got[peer].ev, 0));
        if (cnt)
            HIPCHK(h, hipMemcpy2DAsync(rep + (size_t)h->agg_off[peer] * nsub, rpitch * sizeof(double), got[peer].ptr,
                                       got[peer].pitch * sizeof(double), cnt * sizeof(double), 3,
                                       hipMemcpyDeviceToDevice, st));
    }
    // this rank's reads are issued; its own block may change once every peer's are
    HIPCHK(h, hipEventRecord(C.ev_done, st));
    {
        std::lock_guard<std::mutex> lk(G.mu);
        for (int peer = 0; peer < n; ++peer)
            if (peer != me) G.done[(size_t)me * n + peer] = {C.seq[peer] + 1, nullptr, C.ev_done, 0};
    }
    G.cv.notify_all();
    CHK(wait_posts(G.done, "read completion"));
    for (int peer = 0; peer < n; ++peer) {
        if (peer == me) continue;
        HIPCHK(h, hipStreamWaitEvent(st, got[peer].ev, 0));
        C.seq[peer] += 1;
    }
    return PAMG_OK;
}

// RCCL: one grouped send / recv per peer and plane (an allgatherv of the blocks); a self-peer communicator
// (pamg_comm_init_self) sends its whole level to itself through RCCL, so the transport runs on one GPU
int gather_rccl(pamg_handle *h, const double *local, int64_t lpitch, double *rep, int64_t rpitch, int nsub,
                hipStream_t st) {
    const bool self_peer = !h->vpart.empty();
    const size_t mine = (size_t)h->U * nsub;
    NCCLCHK(h, ncclGroupStart());
    for (int r = 0; r < h->nranks; ++r) {
        if (r == h->rank && !self_peer) continue;   // (copied on the device)
        const size_t cnt = (size_t)(h->agg_off[r + 1] - h->agg_off[r]) * nsub;
        for (int c = 0; c < 3; ++c) {
            if (mine) NCCLQ(h, ncclSend(local + c * lpitch, mine, ncclDouble, r, h->comm->nccl, st));
            if (cnt)
                NCCLQ(h, ncclRecv(rep + c * rpitch + (size_t)h->agg_off[r] * nsub, cnt, ncclDouble, r, h->comm->nccl, st));
        }
    }
    return nccl_group_end(h);
}

// level L's field `local` of every rank into the replica's `rep`
int agg_gather(pamg_handle *h, const double *local, double *rep) {
    const int L = h->p.multi_levels;
    const Level &V = h->lv[L], &R = h->agg->lv[L];
    Span sp(h, PAMG_K_COARSE_GATHER, 24.0 * (double)R.N);   // the whole level arrives (this rank's block by copy)
    const bool self_peer = !h->vpart.empty();
    if (!self_peer && h->U)
        HIPCHK(h, hipMemcpy2DAsync(rep + (size_t)h->agg_off[h->rank] * V.nsub, R.pitch * sizeof(double), local,
                                   V.pitch * sizeof(double), (size_t)h->U * V.nsub * sizeof(double), 3,
                                   hipMemcpyDeviceToDevice, h->stream));
    if (h->comm && h->comm->nccl) return gather_rccl(h, local, V.pitch, rep, R.pitch, V.nsub, h->stream);
    if (h->comm && h->comm->local) return gather_local(h, local, V.pitch, rep, R.pitch, V.nsub, h->stream);
    return PAMG_OK;   // a detached partition (timing probes): its own block only
}

// this rank's block of the replica's level-L fields back into its own level L
int agg_copy_back(pamg_handle *h, bool res) {
    const int L = h->p.multi_levels;
    Level &V = h->lv[L];
    const Level &R = h->agg->lv[L];
    if (!h->U) return PAMG_OK;
    const size_t off = (size_t)h->agg_off[h->vpart.empty() ? h->rank : 0] * V.nsub;
    for (int f = 0; f < 3; ++f) {
        if (f == 2 && !res) continue;
        double *dst = f == 0 ? V.T : f == 1 ? V.TNN : V.RES;
        const double *src = f == 0 ? R.T : f == 1 ? R.TNN : R.RES;
        HIPCHK(h, hipMemcpy2DAsync(dst, V.pitch * sizeof(double), src + off, R.pitch * sizeof(double),
                                   (size_t)h->U * V.nsub * sizeof(double), 3, hipMemcpyDeviceToDevice, h->stream));
    }
    return PAMG_OK;
}

// the reference cycle's coarsest-level work of cycle c (vcycle_face_fused: the restriction-leg call, the
// residual in the call's last cycle, the coarse solve -- or their merged call) on the replica
int agg_coarse_cycle(pamg_handle *h, bool first, bool last) {
    const int L = h->p.multi_levels;
    pamg_handle *r = h->agg;
    if (first) CHK(agg_gather(h, h->lv[L].T, r->lv[L].T));
    CHK(agg_gather(h, h->lv[L].RHS, r->lv[L].RHS));
    CHK(face_pp_level(r, L, last));
    return last ? agg_copy_back(h, true) : PAMG_OK;
}

int smooth_to_tnew(pamg_handle *h, int l, int sweeps);

// the corrected cycle's coarse solve (vcycle_corrected: tnew := 0, n_smooth n_coarse sweeps, tnew := the
// result) on the replica; its result is read by the interpolation into level L - 1
int agg_coarse_corrected(pamg_handle *h) {
    const int L = h->p.multi_levels, ns = h->p.n_smooth;
    pamg_handle *r = h->agg;
    Level &C = r->lv[L];
    CHK(agg_gather(h, h->lv[L].RHS, C.RHS));
    HIPCHK(h, hipMemsetAsync(C.T, 0, 3 * (size_t)C.pitch * sizeof(double), h->stream));   // from zero
    if (ns * h->p.n_coarse > 0 && face_fusable(r, L)) CHK(face_call(r, L, true, ns * h->p.n_coarse, false, false, true));
    else CHK(smooth_to_tnew(r, L, ns * h->p.n_coarse));
    return agg_copy_back(h, false);
}

int vcycle_face_fused(pamg_handle *h, int n) {
    if (h->p.multi_levels >= 2 && h->p.n_smooth >= 2)
        for (int l = 1; l < h->p.multi_levels; ++l)
            if (face_pp_ok(h, l)) return vcycle_face_pp(h, n);
    const int L = h->p.multi_levels, ns = h->p.n_smooth;
    const double rdt = 1 / h->p.dt;
    for (int c = 0; c < n; ++c) {
        const bool last = c + 1 == n;
        for (int l = 1; l <= L; ++l) {   // :323-340
            if (l == L && h->agg) break;   // (the replica runs the coarsest level, below)
            if (l == L && face_coarse_merged(h, last)) break;   // (the call below runs both)
            CHK(face_call(h, l, true, ns, true));
            CHK(restrict_(h, l));
            if (l < L) continue;   // levels < L: get_residual rides on the prolongation-leg call below
            if (!last) continue;   // the coarsest level's: read by nothing, rewritten next cycle (face_pp_level)
            Level &V = h->lv[l];
            h->rhsn_valid = false;
            Span sp(h, PAMG_K_RESIDUAL, 72.0 * (double)V.N + 168.0 * h->U);   // tnew, RHS in, residual out
            HIPCHK(h, launch_face_residual(h->stream, V, h->tov, false, l == 1, rdt, h->slots));
        }
        if (h->agg) CHK(agg_coarse_cycle(h, c == 0, last));   // a partition: the agglomerated coarsest level
        else if (face_coarse_merged(h, last)) CHK(face_call(h, L, true, ns + ns * h->p.n_coarse - 1, true));
        else CHK(face_call(h, L, true, ns * h->p.n_coarse, !last));   // :344-359
        // :363-378; the residual of the restriction leg (:336) is due after the level's call there, and
        // nothing changes level l's tnew, RHS or halo words until this call starts: it computes it
        for (int l = L - 1; l >= 1; --l) CHK(face_call(h, l, true, ns, !last, true));
    }
    h->tnn_level = 1;
    return face_chain_check(h);
}

// the corrected V-cycle (params.cycle = 1; oracle orc_vcycle_corrected):
// the reference's smoother, restrictor and levels with the cycle's defects fixed -- the
// restrictor acts on the fresh residual b - A x, coarse levels start from zero, the prolonged
// correction is added to the iterate the next smoother call starts from. A level's iterate
// after a smoother call is its tnew_nonlin (the last sweep), copied to tnew.
int smooth_to_tnew(pamg_handle *h, int l, int sweeps) {
    Level &L = h->lv[l];
    CHK(smooth(h, l, true, sweeps));
    HIPCHK(h, launch_copy(h->stream, L.TNN, L.T, 3 * L.pitch));
    return PAMG_OK;
}

int residual_corrected(pamg_handle *h, int l) {
    if (h->p.op == 1) return face_residual(h, l, true);
    h->rhsn_valid = false;
    Span sp(h, PAMG_K_RESIDUAL, 72.0 * (double)h->lv[l].N + 168.0 * h->U);
    HIPCHK(h, launch_residual(h->stream, h->lv[l], 1 / h->p.dt, true));
    return PAMG_OK;
}

int vcycle_corrected(pamg_handle *h) {
    const int L = h->p.multi_levels, ns = h->p.n_smooth;
    h->overlap_static_l1 = false;   // the smoother calls rewrite the halo words
    for (int l = 1; l < L; ++l) {
        if (l > 1) HIPCHK(h, hipMemsetAsync(h->lv[l].T, 0, 3 * (size_t)h->lv[l].pitch * sizeof(double), h->stream));
        CHK(smooth_to_tnew(h, l, ns));
        CHK(residual_corrected(h, l));
        CHK(restrict_(h, l));
    }
    Level &C = h->lv[L];
    if (L > 1 && !h->agg) HIPCHK(h, hipMemsetAsync(C.T, 0, 3 * (size_t)C.pitch * sizeof(double), h->stream));   // a coarse level starts from zero
    if (h->agg) {
        CHK(agg_coarse_corrected(h));   // a partition: the agglomerated coarsest level
    } else if (L == 1) {
        CHK(smooth_to_tnew(h, 1, ns));
        CHK(residual_corrected(h, 1));
    } else if (h->p.coarse_solver == 1) {
        CHK(direct_solve(h, L));
    } else {
        CHK(smooth_to_tnew(h, L, ns * h->p.n_coarse));
    }
    for (int l = L - 1; l >= 1; --l) {
        {
            Span sp(h, PAMG_K_PROLONG, 216.0 * (double)h->lv[l + 1].N);
            HIPCHK(h, launch_interp_add(h->stream, h->lv[l], h->lv[l + 1]));
        }
        CHK(smooth_to_tnew(h, l, ns));
    }
    if (L > 1) CHK(residual_corrected(h, 1));   // the fine residual after the cycle
    h->tnn_level = 1;
    return PAMG_OK;
}

// The corrected cycle on the face-coupled operator (op = 1, cycle = 1) with the smoother calls of the levels
// below the coarsest as two-sweep passes (k_face_pp; single domain, face_pp_ok) instead of one launch per
// sweep and a copy: each call runs its n_smooth sweeps from tnew in passes whose last one stores the result
// as tnew (and, in the call's last cycle, as tnew_nonlin too -- inside the call tnew_nonlin is overwritten
// before any read); the coarsest level's calls stay one chain launch (face_call). The passes do not publish
// halo words between sweeps (they read the neighbours' iterate itself), and no operation of the cycle reads
// t_overlap but the residuals, each of which refreshes the words from its level's tnew first (face_residual)
// -- as does the per-step sequence's last operation, the fine residual after the cycle, which only the
// call's last cycle runs here (the next cycle's first residual rewrites it unread, and its words). Every
// sub-element's arithmetic is face_apply's: the state after the call is bitwise vcycle_corrected's
// (tests/test_face_operator.py). PAMG_FACE_CORR_PP=0 keeps the per-step sequence (A/B).
bool face_corrected_pp_ok(pamg_handle *h) {
    const char *ev = getenv("PAMG_FACE_CORR_PP");   // read per call: tests switch it within a process
    const bool off = ev && atoi(ev) == 0;
    if (off || !(h->p.op == 1 && h->p.cycle == 1 && h->p.fused && h->p.coarse_solver == 0 && h->p.n_smooth >= 3 &&
                 h->p.multi_levels >= 2))
        return false;
    for (int l = 1; l < h->p.multi_levels; ++l)
        if (face_pp_ok(h, l)) return true;
    return false;
}

// one smoother call of the corrected cycle on level l < L: tnew := the result of n_smooth sweeps from tnew;
// streaming levels only (face_pp_ok): from_zero -- from a zero iterate (the cycle's memset of a coarse level
// folded: the first pass reads no iterate), interp -- from tnew plus the prolonged coarse correction (the
// cycle's interp_add folded into the first pass, which adds it to every value it loads: bitwise the
// correction stored and read back; the corrected iterate itself is overwritten unread by the call's result)
int face_corr_call(pamg_handle *h, int l, bool last, bool from_zero = false, bool interp = false) {
    const int ns = h->p.n_smooth;
    if (!face_pp_ok(h, l)) {
        if (from_zero || interp) { h->err = "internal: a folded face call on a level that does not stream"; return PAMG_ERR_STATE; }
        CHK(smooth_to_tnew(h, l, ns));
        return PAMG_OK;
    }
    h->tnn_level = l;
    h->overlap_static_l1 = false;
    std::vector<PPPass> plan;
    CHK(face_pp_plan(h, l, ns, from_zero ? nullptr : h->lv[l].T, {}, last ? 3 : 2, plan));
    plan[0].interp = interp;
    for (const PPPass &q : plan) CHK(face_pp_emit(h, l, q));
    return PAMG_OK;
}

// the corrected cycle's get_residual and restrictor of a level l < L (:336-338) as one sweep-less k_face_pp pass
// (res 3): the residual RHS - A tnew from the neighbours' iterate itself, restricted straight into RHS_{l+1}
// (k_restrict_tile's arithmetic). The residual is stored only where the state keeps it: level 1's is rewritten
// by the fine residual after the cycle (the call's last cycle); a coarser level's is kept from the call's last
// cycle. The halo words the per-step residual refreshes first are rewritten, unread, by that same fine residual
// (every coarser level's words are a subset of level 1's slots).
int face_res_restrict(pamg_handle *h, int l, bool last) {
    Level &L = h->lv[l];
    h->rhsn_valid = false;
    h->overlap_static_l1 = false;
    const bool store = l > 1 && last;
    Span sp(h, PAMG_K_RESIDUAL, (48.0 + (store ? 24.0 : 0.0)) * (double)L.N + 24.0 * (double)h->lv[l + 1].N + 168.0 * h->U);
    PPCoarse pc;
    pc.coarse = &h->lv[l + 1];
    pc.rhsc = h->lv[l + 1].RHS;
    pc.res_store = store;
    HIPCHK(h, launch_face_pp(h->stream, L, 1, L.T, nullptr, nullptr, nullptr, h->p.solver == 3, l == 1, 1 / h->p.dt, 3,
                             nullptr, &pc));
    return PAMG_OK;
}

int vcycle_corrected_face_pp(pamg_handle *h, int n) {
    const int L = h->p.multi_levels, ns = h->p.n_smooth;
    h->overlap_static_l1 = false;
    // PAMG_FACE_RR=0 (A/B): the residual and the restrictor as their own launches; PAMG_FACE_FOLD=0: a coarse
    // level's memset and the interpolation as their own launches
    const char *rr_env = getenv("PAMG_FACE_RR"), *fold_env = getenv("PAMG_FACE_FOLD");
    const bool rr = !(rr_env && atoi(rr_env) == 0), fold = !(fold_env && atoi(fold_env) == 0);
    for (int c = 0; c < n; ++c) {
        const bool last = c + 1 == n;
        for (int l = 1; l < L; ++l) {
            const bool fz = l > 1 && fold && face_pp_ok(h, l);
            if (l > 1 && !fz) HIPCHK(h, hipMemsetAsync(h->lv[l].T, 0, 3 * (size_t)h->lv[l].pitch * sizeof(double), h->stream));
            CHK(face_corr_call(h, l, last, fz));
            if (rr && face_pp_ok(h, l)) {
                CHK(face_res_restrict(h, l, last));
            } else {
                CHK(residual_corrected(h, l));
                CHK(restrict_(h, l));
            }
        }
        Level &C = h->lv[L];
        HIPCHK(h, hipMemsetAsync(C.T, 0, 3 * (size_t)C.pitch * sizeof(double), h->stream));   // from zero
        if (fold && ns * h->p.n_coarse > 0 && face_fusable(h, L)) {
            CHK(face_call(h, L, true, ns * h->p.n_coarse, false, false, true));   // tnew := the result: the final stores
        } else {
            CHK(smooth_to_tnew(h, L, ns * h->p.n_coarse));
        }
        for (int l = L - 1; l >= 1; --l) {
            if (fold && face_pp_ok(h, l)) {
                CHK(face_corr_call(h, l, last, false, true));
                continue;
            }
            {
                Span sp(h, PAMG_K_PROLONG, 216.0 * (double)h->lv[l + 1].N);
                HIPCHK(h, launch_interp_add(h->stream, h->lv[l], h->lv[l + 1]));
            }
            CHK(face_corr_call(h, l, last));
        }
        if (last) CHK(residual_corrected(h, 1));   // the fine residual after the cycle
    }
    h->tnn_level = 1;
    return face_chain_check(h);
}

// the corrected cycle as one resident launch per pamg_vcycle call (pamg_vcycle_impl.h k_vc_corr): the
// call's cycles with every level of a tile on-chip, the state stored once at the end -- bitwise the
// per-step sequence above (tests/test_corrected.py). The halo words of the state are the last smoother
// call's, level 1's post-smoothing call of the last cycle (every coarser level writes a subset of its
// slots before it): its tnew words are written by the launch, the words constant within a time step by
// k_overlap_static, the remote ones exchanged after the call (halo_exchange = 0). fused = 0 keeps the per-step
// sequence.
int call_schedule(pamg_handle *h);
bool corrected_resident_ok(pamg_handle *h) {
    return h->p.cycle == 1 && h->p.fused != 0 && h->p.op == 0 && h->p.coarse_solver == 0 && h->p.solver != 2 &&
           h->p.halo_exchange == 0 && h->p.n_smooth > 0 && call_schedule(h) == 3 &&
           vcycle_corrected_supported(h->p.n_split, h->p.multi_levels);
}

// algorithmic HBM bytes of the corrected resident call: level 1 reads tnew and RHS and writes tnew,
// tnew_nonlin and the residual (120 B); a level between writes RHS, residual, tnew, tnew_nonlin (96 B);
// the coarsest RHS, tnew, tnew_nonlin (72 B); the operator words (104 B per un_ele and level)
double vcycle_corr_bytes(pamg_handle *h) {
    const int L = h->p.multi_levels;
    double b = 120.0 * h->lv[1].N;
    for (int l = 2; l <= L; ++l) b += (l < L ? 96.0 : 72.0) * h->lv[l].N;
    return b + 104.0 * h->U * L;
}

int overlap_static_once(pamg_handle *h);
int vcycle_corrected_resident(pamg_handle *h, int n) {
    if (n <= 0) return PAMG_OK;
    const int L = h->p.multi_levels;
    HaloPlan &P1 = h->lv[1].halo;
    CHK(overlap_static_once(h));
    const int buf = P1.d_send_b ? 1 - P1.send_cur : 0;
    if (h->sent_pending[buf]) {   // the exchange that read this buffer
        HIPCHK(h, hipStreamWaitEvent(h->stream, h->ev_sent[buf], 0));
        h->sent_pending[buf] = false;
    }
    h->rhsn_valid = false;   // residuals and coarse RHS rewritten (RHSN does not follow them)
    {
        Span sp(h, PAMG_K_VCYCLE_CORR, vcycle_corr_bytes(h));
        HIPCHK(h, launch_vcycle_corrected(h->stream, h->lv, L, h->U, h->p.n_split, h->p.n_smooth, h->p.n_coarse,
                                          1 / h->p.dt, h->tov, h->tovo, P1.send_buf(buf), h->lv[2].RHSN, PAMG_KEEP_ALL, n));
    }
    h->tnn_level = 1;
    CHK(halo_async(h, buf));
    return join_comm(h);
}

// n V-cycles as two fused launches each (pamg_vcycle.hip)
// pipelined-call schedule (pamg_set_call_schedule)
// 0 automatic: the resident form where it applies (two levels or more, the halo words exchanged
// once per call), else one launch per cycle (one GPU) or two tile streams (a partition)
int call_schedule(pamg_handle *h) {
    const int s = h->call_schedule;
    if (s) return s;
    if (vcycle_resident_supported(h->p.n_split, h->p.multi_levels)) return 3;
    return h->nranks > 1 ? 2 : 1;
}

// the fused forms of the V-cycle apply; Richardson (solver 2) has its update only in the resident
// call (pamg_vcycle.hip k_vc_res with StcR), so it is fused there and nowhere else
bool fused_ok(pamg_handle *h) {
    const int L = h->p.multi_levels;
    if (!(h->p.fused && h->p.cycle == 0 && h->p.coarse_solver == 0 && h->p.op == 0 &&
          vcycle_fusable(h->lv, L, h->p.n_split, h->p.solver, h->p.halo_mode, h->p.n_smooth)))
        return false;
    if (h->p.solver != 2) return true;
    return h->p.fused == 3 && call_schedule(h) == 3 && !h->coarse_ahead && vcycle_resident_supported(h->p.n_split, L);
}


// once per time step: the level-1 halo words the cycle's last smoother call leaves constant
// (t_overlap_old, the boundary words, the told halves of the send entries -- into both send buffers)
int overlap_static_once(pamg_handle *h) {
    if (h->overlap_static_l1) return PAMG_OK;
    HaloPlan &P1 = h->lv[1].halo;
    CHK(join_comm(h));
    HIPCHK(h, launch_overlap_static(h->stream, h->lv[1], h->U, h->tov, h->tovo, nullptr, h->told_halo_stale_l1));
    h->told_halo_stale_l1 = false;
    if (P1.d_send_b) HIPCHK(h, launch_overlap_static(h->stream, h->lv[1], h->U, h->tov, h->tovo, P1.d_send_b));
    h->overlap_static_l1 = true;
    return PAMG_OK;
}

// dead_after (pamg_run, every step but the last): the next call rewrites the fields this one
// leaves for an observer -- level 1's residual and tnew_nonlin, the coarse levels' RHS and
// residual, the halo words -- before any read (nothing reads t_overlap, the next step's first
// restrictor reads level 2's RHSN, which is stored), so the pipelined schedule skips them
// and the exchange of the halo words too
// steps > 1: the resident schedule runs `steps` time steps of n cycles in one launch (pamg_run;
// the call starts the first step, rhs_pending)
int vcycle_fused(pamg_handle *h, int n, bool dead_after, int steps = 1) {
    const int L = h->p.multi_levels, ns = h->p.n_smooth;
    const double rdt = 1 / h->p.dt;
    HaloPlan &P1 = h->lv[1].halo;
    const bool two = P1.d_send_b != nullptr;   // remote peers: pack into alternate buffers
    if (!h->rhsn_valid) {   // residuals changed outside the fused cycle: restrict them afresh
        for (int l = 1; l < L; ++l)
            HIPCHK(h, launch_restrict(h->stream, h->lv[l], h->lv[l + 1], h->U, h->lv[l + 1].RHSN));
        h->rhsn_valid = true;
    }
    // once per time step: the halo words the cycle's last smoother leaves constant (into both
    // send buffers); when this call starts a pamg_run step whose told and RHS its first level-1
    // launch computes (rhs_pending), after that launch, as it reads told
    auto overlap_static = [&]() -> int { return overlap_static_once(h); };
    const bool rhs_first = h->rhs_pending;
    h->rhs_pending = false;
    if (!rhs_first) CHK(overlap_static());
    // fused = 2: the coarse launch of cycle c (levels 2..L, fp64-issue-bound) runs on stream_c
    // beside the level-1 launch of cycle c (HBM-bound). Their only shared data is level 2's
    // RHSN, read by the coarse launch and written by the level-1 launch: double-buffered,
    // so coarse(c) waits for level 1(c-1) (its RHS) and level 1(c) waits for coarse(c-1)
    // (the reader of the buffer it overwrites). The level-1 launch's prolongator (:370)
    // reads level 2's tnew, which coarse(c) may be rewriting: its result is dead (:550,
    // SURVEY.md A3 iv) and never stored, so no state depends on the order.
    const bool conc = h->p.fused == 2 && L > 1;
    // fused = 3: coarse(1), then [level 1 (c) + coarse levels (c+1)] for c < n, then level 1 (n)
    // (pamg_vcycle.hip, "pipelined tail"): nothing outside the call sees the coarse levels
    // one cycle ahead, and the last launch brings level 1 (and level 2's RHSN) level with them
    const bool pipe = h->p.fused == 3 && L > 1;
    Level &L2 = h->lv[2];
    // pipelined, halo exchanged once per call: the tiles are independent for the whole call
    // (every operation is local to an un_ele, the halo words have no reader inside it), so two
    // halves of them can run their launch sequences on two streams, each launch's drain
    // overlapped by the other half's stream (schedule 2). Measured (scripts/ab_probe.py, profiles/r01_v16_tile_streams.txt):
    // N = 4 partition 0.0404 -> 0.0339 ms per cycle, N = 8 0.0208 -> 0.0202, n_split = 3
    // 0.0128 -> 0.0114, full mesh 0.1319 -> 0.1290. Automatic on partitions only: on one GPU
    // the bench's per-launch events time launches, which schedule 2 overlaps.
    //
    // pamg_set_call_schedule(h, s): 0 automatic (3 where it applies, else 2 on a partition of
    // a multi-rank run, 1 on one GPU), 1 one launch per cycle, 2 two tile streams, 3 resident
    // (below). (Round 1 tried a persistent
    // form of the pipelined launch and dropped it at 128 VGPRs with spills; the resident form
    // fits -- its final-cycle stores are peeled out of the cycle loop and its loop is
    // unswitched by wave role, pamg_vcycle.hip k_vc_res / k_vc_resb.)
    const int tile = vcycle_tile_un_eles(h->p.n_split);
    const int ntiles = (h->U + tile - 1) / tile;
    const int sched = call_schedule(h);
    // schedule 3, resident: the call's n cycles in one launch (pamg_vcycle.hip k_vc_res), every
    // tile's state on-chip between them; the final-cycle stores as the pipelined schedule makes
    // them (the call's last launch stores all, or inside pamg_run the fields the next step reads)
    if (steps > 1 && !(pipe && n >= 1 && sched == 3 && h->p.halo_exchange == 0 && !h->coarse_ahead && rhs_first &&
                       vcycle_resident_run_supported(h->p.n_split, L))) {
        h->err = "internal: a resident run outside the resident schedule";
        return PAMG_ERR_STATE;
    }
    if (h->p.solver == 2 && n >= 1 &&
        !(pipe && sched == 3 && !h->coarse_ahead && vcycle_resident_supported(h->p.n_split, L))) {
        h->err = "internal: Richardson outside the resident call";
        return PAMG_ERR_STATE;
    }
    if (pipe && n >= 1 && sched == 3 && !h->coarse_ahead && vcycle_resident_supported(h->p.n_split, L)) {
        const int buf = two ? 1 - P1.send_cur : 0;
        if (h->sent_pending[buf]) {
            HIPCHK(h, hipStreamWaitEvent(h->stream, h->ev_sent[buf], 0));
            h->sent_pending[buf] = false;
        }
        const bool rhsf = rhs_first;
        const int kt = rhsf && !dead_after ? PAMG_KEEP_TOLD : 0;
        // inside pamg_run (dead_after) the halo words die unread too -- unless every cycle's are exchanged
        const bool hx = h->p.halo_exchange == 1;
        const int keep = (dead_after ? kPipeKeep | (hx ? PAMG_KEEP_HALO : 0) : PAMG_KEEP_ALL) | kt;
        if (kt) CHK(join_comm(h));   // the send buffers' told halves are rewritten
        // halo_exchange = 1: every cycle's words are exchanged. Cycles 0 .. n-2 pack the tnew words
        // of their remote entries into level 1's ring (k_vc_res / k_vc_resb with XC) and publish
        // each completed cycle on xc_sig; the comm stream waits for cycle c's count
        // (hipStreamWaitValue64) and exchanges it (exchange_ring) while the launch runs on; the last
        // cycle's words (6 per entry, with told) go as in the plain call, after the launch
        const bool xc = hx && n >= 2 && !P1.remote.empty();
        if (xc && (rhsf || steps != 1)) {
            h->err = "internal: a per-cycle exchange inside a resident time step";
            return PAMG_ERR_STATE;
        }
        if (xc) {
            CHK(xc_setup(h, n));
            HIPCHK(h, hipMemsetAsync(h->xc_done, 0, (size_t)(n - 1) * sizeof(unsigned), h->stream));
            {
                Span sp(h, PAMG_K_VCYCLE_RES, vcycle_res_bytes(h, keep, false) + 24.0 * (n - 1) * P1.remote.size());
                HIPCHK(h, launch_vcycle_resident_xc(h->stream, h->lv, L, h->U, h->p.n_split, ns, h->p.n_coarse, rdt,
                                                    h->tov, h->tovo, P1.send_buf(buf), L2.RHSN, keep, n, P1.d_ring,
                                                    3 * (int64_t)P1.remote.size(), h->xc_done, h->xc_sig));
            }
            if (h->comm && !P1.peers.empty())
                for (int c = 0; c + 1 < n; ++c) {
                    HIPCHK(h, hipStreamWaitValue64(h->stream_comm, h->xc_sig, h->xc_sig_base + c + 1,
                                                   hipStreamWaitValueGte));
                    CHK(exchange_ring(h, c, h->stream_comm));
                }
            h->xc_sig_base += (unsigned long long)(n - 1);
        } else {
            // the per-call exchange, started early: the call's halo words are final once a tile has run its
            // last cycle, so the tiles with remote faces run first (tile order), count their ends, and the
            // last of them raises xc_sig; the comm stream waits on it and exchanges while the other tiles'
            // rounds run (the exchange reads only their send words and writes only the remote slots of
            // t_overlap / t_overlap_old, which no tile of the launch writes). A call that starts a time step
            // (RHSF) writes the send buffers' told halves itself and exchanges after the launch.
            const bool xe = !rhsf && !dead_after && steps == 1 && h->comm && !P1.peers.empty();
            EarlyXc X{};
            if (xe) {
                // the counter is never reset (a memset before the launch delays it by a few us): this call's
                // remote tiles complete it at the running total
                CHK(xe_setup(h));
                h->xe_total += (unsigned)h->xe_nremote;
                X = EarlyXc{h->xe_map, h->xe_done, h->xe_total, h->xc_sig};
            }
            const bool diag = xe && (h->timing.mask & (1u << PAMG_K_HALO_EARLY));
            if (diag) {
                for (auto &e : h->xe_ev)
                    if (!e) HIPCHK(h, hipEventCreate(&e));
                HIPCHK(h, hipEventRecord(h->xe_ev[0], h->stream));
            }
            {
                Span sp(h, rhsf ? PAMG_K_VCYCLE_RES_RHSF : PAMG_K_VCYCLE_RES, vcycle_res_bytes(h, keep, rhsf));
                HIPCHK(h, launch_vcycle_resident(h->stream, h->lv, L, h->U, h->p.n_split, ns, h->p.n_coarse, rdt, h->tov,
                                                 h->tovo, P1.send_buf(buf), L2.RHSN, keep, rhsf,
                                                 two ? P1.send_buf(1 - buf) : nullptr, n, steps, xe ? &X : nullptr));
            }
            if (xe) {
                if (diag) HIPCHK(h, hipEventRecord(h->xe_ev[3], h->stream));
                HIPCHK(h, hipStreamWaitValue64(h->stream_comm, h->xc_sig, h->xc_sig_base + 1, hipStreamWaitValueGte));
                h->xc_sig_base += 1;
                if (diag) HIPCHK(h, hipEventRecord(h->xe_ev[1], h->stream_comm));
                {
                    Span sp(h, PAMG_K_HALO_EARLY, 2.0 * 48.0 * (double)(P1.remote.size() + P1.recv_dst.size()),
                            h->stream_comm);
                    CHK(exchange(h, 1, buf, h->stream_comm));
                }
                if (diag) {
                    HIPCHK(h, hipEventRecord(h->xe_ev[2], h->stream_comm));
                    h->xe_ev_valid = true;
                }
                HIPCHK(h, hipEventRecord(h->ev_sent[buf], h->stream_comm));
                h->sent_pending[buf] = true;
                P1.send_cur = buf;
                h->tnn_level = 1;
                // the join of `stream` behind the exchange is left to the next operation that needs it (settle,
                // at the entry of every other call; the next resident call waits only for the exchange that
                // read the send buffer it packs): a barrier packet behind the launch cost ~5-8 us of a 20-cycle
                // call at an N = 8 rank's shape (profiles/r05_i_xe_join.txt); pamg_synchronize waits for both
                return PAMG_OK;
            }
        }
        if (rhsf) {
            h->overlap_static_l1 = kt != 0;
            h->told_halo_stale_l1 = kt == 0;
        }
        h->tnn_level = 1;
        if (dead_after && !hx) {
            P1.send_cur = buf;
            return join_comm(h);
        }
        CHK(halo_async(h, buf));
        return join_comm(h);
    }
    if (pipe && n > 1 && sched == 2 && h->p.halo_exchange == 0 && ntiles >= 2 && !h->coarse_ahead) {
        const int buf = two ? 1 - P1.send_cur : 0;
        if (h->sent_pending[buf]) {
            HIPCHK(h, hipStreamWaitEvent(h->stream, h->ev_sent[buf], 0));
            h->sent_pending[buf] = false;
        }
        const int mid = (ntiles / 2) * tile;
        HIPCHK(h, hipEventRecord(h->ev_fine, h->stream));
        HIPCHK(h, hipStreamWaitEvent(h->stream_c, h->ev_fine, 0));
        // launches alternate between the halves so that each stream always has the next one queued
        const hipStream_t st[2] = {h->stream, h->stream_c};
        // the first coarse launch's RHS and residual are rewritten by the first pipelined one
        const int ck = kPipeKeep & PAMG_KEEP_COARSE;
        const int ua[2] = {0, mid}, ub[2] = {mid, h->U};
        const int kf = dead_after ? kPipeKeep : PAMG_KEEP_ALL;   // the call's last level-1 launch
        for (int q = 0; q < 2; ++q) {
            Span sp(h, PAMG_K_VCYCLE_COARSE, vcycle_coarse_bytes(h, ck) * (ub[q] - ua[q]) / h->U, st[q]);
            HIPCHK(h, launch_vcycle_coarse(st[q], h->lv, L, h->U, h->p.n_split, ns, h->p.n_coarse, rdt, h->tov,
                                           h->tovo, L2.RHSN, ua[q], ub[q], ck));
        }
        for (int c = 0; c < n; ++c) {
            const bool pc = c + 1 < n;
            const int keep = pc ? kPipeKeep | (c + 2 == n && !dead_after ? PAMG_KEEP_COARSE : 0) : kf;
            for (int q = 0; q < 2; ++q) {
                const double f = (double)(ub[q] - ua[q]) / h->U;
                Span sp(h, pc ? PAMG_K_VCYCLE_PIPE : PAMG_K_VCYCLE,
                        f * (pc ? vcycle_pipe_bytes(h, keep) : vcycle_fine_bytes(h, keep)), st[q]);
                HIPCHK(h, launch_vcycle_fine(st[q], h->lv, L, h->U, h->p.n_split, ns, h->p.n_coarse, rdt, h->tov,
                                             h->tovo, P1.send_buf(buf), L2.RHSN, pc, keep, ua[q], ub[q]));
            }
        }
        HIPCHK(h, hipEventRecord(h->ev_coarse, h->stream_c));
        HIPCHK(h, hipStreamWaitEvent(h->stream, h->ev_coarse, 0));
        h->tnn_level = 1;
        if (dead_after) {
            P1.send_cur = buf;
            return join_comm(h);
        }
        CHK(halo_async(h, buf));
        return join_comm(h);
    }
    if (conc) {
        HIPCHK(h, hipEventRecord(h->ev_fine, h->stream));   // everything issued before this call
    }
    // pamg_run: a step's last launch may have run this call's first coarse cycle already
    // (into_next below); else its RHS and residual stores are rewritten by the first
    // pipelined launch if n > 1
    if (pipe && n > 0 && !h->coarse_ahead) {
        const int ck = (n > 1 || dead_after) ? kPipeKeep & PAMG_KEEP_COARSE : PAMG_KEEP_ALL;
        Span sp(h, PAMG_K_VCYCLE_COARSE, vcycle_coarse_bytes(h, ck));
        HIPCHK(h, launch_vcycle_coarse(h->stream, h->lv, L, h->U, h->p.n_split, ns, h->p.n_coarse, rdt, h->tov,
                                       h->tovo, L2.RHSN, 0, -1, ck));
    }
    h->coarse_ahead = false;
    // pamg_run, every step but the last: the call's last level-1 launch is a pipelined one too,
    // carrying the next step's first coarse cycle -- it depends on this call's last residual
    // (:336) and on the coarse levels' own state only, not on begin_timestep (level 1) -- so
    // each step saves its separate coarse launch
    const bool into_next = pipe && dead_after && h->p.halo_exchange == 0;
    for (int c = 0; c < n; ++c) {
        const int buf = two ? 1 - P1.send_cur : 0;
        if (h->sent_pending[buf]) {   // the exchange that read this buffer two cycles ago
            HIPCHK(h, hipStreamWaitEvent(h->stream, h->ev_sent[buf], 0));
            h->sent_pending[buf] = false;
        }
        double *rhsn_w = conc ? (L2.RHSN == L2.RHSN_alt ? L2.T + 15 * L2.pitch : L2.RHSN_alt) : L2.RHSN;
        if (conc) {
            HIPCHK(h, hipStreamWaitEvent(h->stream_c, h->ev_fine, 0));
            if (c > 0) HIPCHK(h, hipStreamWaitEvent(h->stream, h->ev_coarse, 0));
        }
        if (L > 1 && !pipe) {   // levels 2..L first: the prolongator of level 1 reads their final tnew
            const hipStream_t sc = conc ? h->stream_c : h->stream;
            Span sp(h, PAMG_K_VCYCLE_COARSE, vcycle_coarse_bytes(h), sc);
            HIPCHK(h, launch_vcycle_coarse(sc, h->lv, L, h->U, h->p.n_split, ns, h->p.n_coarse, rdt, h->tov,
                                           h->tovo, L2.RHSN));
            if (conc) HIPCHK(h, hipEventRecord(h->ev_coarse, h->stream_c));
        }
        {
            const bool pc = pipe && (c + 1 < n || into_next);   // also the coarse levels of cycle c + 1
            // its stores that the rest of the call overwrites unread are skipped: level 1's
            // residual and tnew_nonlin always (the call's last launch is k_vc_fine, which stores
            // them), the coarse levels' RHS and residual unless they reach their final cycle
            // here, the halo words unless every cycle's are exchanged
            const bool dead = pipe && dead_after && h->p.halo_exchange == 0;
            const int keep = c + 1 == n && into_next ? kPipeKeep | (n == 1 ? PAMG_KEEP_COARSE : 0)
                             : pc ? kPipeKeep | (c + 2 == n && !dead ? PAMG_KEEP_COARSE : 0) |
                                        (h->p.halo_exchange == 1 ? PAMG_KEEP_HALO : 0)
                                  : (dead && c + 1 == n ? kPipeKeep : PAMG_KEEP_ALL);
            // rhs_first: this launch also starts the time step -- told := tnew and level 1's RHS
            // (k_rhs's work: +48 B stored, 24 B of RHS not read per level-1 sub-element)
            // (+24 B of s' read and 24 B of RHS stored per level-1 sub-element, the RHS read
            // saved; kKeepTold, the step the next one does not overwrite: told stored and the
            // step's constant halo words written, k_overlap_static's work)
            const bool rhsf = rhs_first && c == 0;
            if (rhsf && !pc) { h->err = "internal: time-step start on a non-pipelined launch"; return PAMG_ERR_STATE; }
            const int kt = rhsf && !dead_after ? PAMG_KEEP_TOLD : 0;
            Span sp(h, rhsf ? PAMG_K_VCYCLE_RHSF : pc ? PAMG_K_VCYCLE_PIPE : PAMG_K_VCYCLE,
                    (pc ? vcycle_pipe_bytes(h, keep) : vcycle_fine_bytes(h, keep)) +
                        (rhsf ? (kt ? 48.0 : 24.0) * h->lv[1].N : 0.0));
            if (kt) CHK(join_comm(h));   // the send buffers' told halves are rewritten
            HIPCHK(h, launch_vcycle_fine(h->stream, h->lv, L, h->U, h->p.n_split, ns, h->p.n_coarse, rdt, h->tov,
                                         h->tovo, P1.send_buf(buf), L > 1 ? rhsn_w : nullptr, pc, keep | kt, 0, -1,
                                         rhsf, two ? P1.send_buf(1 - buf) : nullptr));
            if (rhsf) {
                // kKeepTold: the launch wrote what k_overlap_static would (from told in registers);
                // else told and those words are dead until the next step rewrites them
                h->overlap_static_l1 = kt != 0;
                h->told_halo_stale_l1 = kt == 0;
            }
            if (conc) HIPCHK(h, hipEventRecord(h->ev_fine, h->stream));
        }
        if (L > 1) L2.RHSN = rhsn_w;   // the next cycle's level-2 RHS
        h->tnn_level = 1;
        // every halo word of the cycle was written by the level-1 launch (its remote ones
        // packed into `buf`); the next cycle rewrites every one of them and nothing reads
        // t_overlap in between: halo_exchange = 0 exchanges the last cycle's words only,
        // 1 every cycle's, in flight during the next one
        if (h->p.halo_exchange == 1 || (c + 1 == n && !(pipe && dead_after))) CHK(halo_async(h, buf));
        else if (c + 1 == n) P1.send_cur = buf;
    }
    h->coarse_ahead = into_next && n > 0;
    if (conc && n > 0) HIPCHK(h, hipStreamWaitEvent(h->stream, h->ev_coarse, 0));   // join
    return join_comm(h);
}

// the replica of the coarsest level for op = 1 on a partition (agg_coarse_cycle); PAMG_FACE_AGG=0 (read here, at
// upload): none -- the partition then runs its coarsest calls one launch per sweep, exchanging between sweeps
int agg_create(pamg_handle *h, int U, const double *X, const int *region, const int *neig, const int *fneig,
               const int *dir) {
    const char *e = getenv("PAMG_FACE_AGG");
    const int L = h->p.multi_levels;
    if (h->coarse_only || h->p.op != 1 || L < 2 || (h->nranks == 1 && h->vpart.empty()) || (e && atoi(e) == 0))
        return PAMG_OK;
    // only a level the persistent chain holds: that is what makes the whole level cost every rank no more than its
    // own part did (latency-bound sweeps); a larger coarsest level stays partitioned, one launch per sweep
    if (!h->cus) {
        int n = 0;
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, h->device) != hipSuccess || n <= 0) n = 1;
        h->cus = n;
    }
    if (!face_chain_fits(1 << (2 * (h->p.n_split - L + 1)), U, h->cus)) return PAMG_OK;
    // the replica's numbering: rank 0's un_eles (ascending global id), then rank 1's, ... (a self-peer
    // communicator: one block, the global order)
    std::vector<int> order;
    order.reserve(U);
    h->agg_off.assign(1, 0);
    if (h->nranks == 1) {
        for (int g = 0; g < U; ++g) order.push_back(g);
        h->agg_off.push_back(U);
    } else {
        for (int r = 0; r < h->nranks; ++r) {
            for (int g = 0; g < U; ++g)
                if (h->owner[g] == r) order.push_back(g);
            h->agg_off.push_back((int)order.size());
        }
    }
    std::vector<int> pnew(U);
    for (int i = 0; i < U; ++i) pnew[order[i]] = i;
    std::vector<double> Xp(6 * (size_t)U);
    std::vector<int> regp(U), neigp(3 * (size_t)U), fneigp(3 * (size_t)U), dirp(3 * (size_t)U);
    for (int i = 0; i < U; ++i) {
        const int g = order[i];
        for (int c = 0; c < 6; ++c) Xp[6 * (size_t)i + c] = X[6 * (size_t)g + c];
        regp[i] = region[g];
        for (int f = 0; f < 3; ++f) {
            const int nb = neig[3 * (size_t)g + f];
            neigp[3 * (size_t)i + f] = nb >= 1 ? pnew[nb - 1] + 1 : nb;
            fneigp[3 * (size_t)i + f] = fneig[3 * (size_t)g + f];
            dirp[3 * (size_t)i + f] = dir[3 * (size_t)g + f];
        }
    }
    // the replica works on this handle's streams (its chains are ordered with the cycle) and creates none of its
    // own but the chain gates' fallback stream, on first use: a process then holds the four streams of a
    // single-domain handle, one per hardware queue (GPU_MAX_HW_QUEUES = 4), so the fallback never waits behind
    // the gate it opens
    auto *r = new pamg_handle;
    r->p = h->p;
    r->device = h->device;
    r->stream = h->stream;
    r->stream_comm = h->stream_comm;
    r->stream_c = h->stream_c;
    r->borrowed_stream = true;
    r->coarse_only = true;
    r->tparent = h;
    r->cus = h->cus;
    const int rc = pamg_upload_mesh(r, U, Xp.data(), regp.data(), neigp.data(), fneigp.data(), dirp.data());
    if (rc != PAMG_OK) {
        h->err = "coarse replica: " + r->err;
        (void)pamg_destroy(r);
        return rc;
    }
    h->agg = r;
    return PAMG_OK;
}

// the communicator (blocking: see nccl_settle); a failure binds nothing to the handle
int nccl_init(pamg_handle *h, ncclComm_t *out, int nranks, ncclUniqueId uid, int rank) {
    *out = nullptr;
    ncclComm_t nc = nullptr;
    const ncclResult_t r = ncclCommInitRank(&nc, nranks, uid, rank);
    if (r != ncclSuccess) {
        h->err = "ncclCommInitRank (rank " + std::to_string(rank) + " of " + std::to_string(nranks) + "): " +
                 ncclGetErrorString(r);
        if (nc) (void)ncclCommAbort(nc);
        return PAMG_ERR_COMM;
    }
    *out = nc;
    return PAMG_OK;
}

void nccl_release(ncclComm_t c) { (void)ncclCommDestroy(c); }

void free_levels(pamg_handle *h) {
    for (int l = 1; l <= kMaxLevels; ++l) {
        Level &L = h->lv[l];
        dev_free(L.T); dev_free(L.stc); dev_free(L.Ainv); dev_free(L.subinfo); dev_free(L.d_pos); dev_free(L.blocks);
        dev_free(L.fnb); dev_free(L.fface); dev_free(L.fsx); dev_free(L.cpos); dev_free(L.gtab); dev_free(L.cnb); dev_free(L.gpat);
        dev_free(L.chain_nb_off); dev_free(L.chain_nb_list); dev_free(L.chain_flags);
        dev_free(L.halo.d_local); dev_free(L.halo.d_bc); dev_free(L.halo.d_remote); dev_free(L.halo.d_recv_dst);
        dev_free(L.halo.d_send); dev_free(L.halo.d_send_b); dev_free(L.halo.d_recv);
        dev_free(L.halo.d_ring); dev_free(L.halo.d_recv3);
        dev_free(L.halo.d_hface); dev_free(L.halo.d_hsub); dev_free(L.halo.d_bcv); dev_free(L.halo.d_bpos);
        dev_free(L.halo.d_surf); dev_free(L.halo.d_told_halo);
        L = Level();
    }
    dev_free(h->geo1); dev_free(h->tov); dev_free(h->tovo); dev_free(h->tov_b);
    h->geo1 = h->tov = h->tovo = h->tov_b = nullptr;
    dev_free(h->wave_order); dev_free(h->wave_neig); dev_free(h->wave_flags); dev_free(h->wave_gran);
    h->wave_order = h->wave_neig = nullptr;
    h->wave_flags = nullptr;
    h->wave_gran = nullptr;
    h->wave_band = -1;
    dev_free(h->xe_map);
    h->xe_map = nullptr;
    h->xe_nremote = -1;
    h->mesh_ready = false;
}

}  // namespace

extern "C" {

int pamg_version(void) { return 100; }

void pamg_default_params(pamg_params *p) {
    std::memset(p, 0, sizeof *p);
    p->n_split = 1;          // :118
    p->multi_levels = 1;     // main.F90:46-47
    p->n_smooth = 4;
    p->n_coarse = 15;        // :351
    p->solver = 3;
    p->device = 0;
    p->dt = 1. * 0.0000125;  // CFL*dx, :133
    p->k = 1.;               // :136
    p->omega = 0.8;          // :140
    p->theta = 1.;           // :117
    p->halo_mode = 0;
    p->fused = 3;
}

int pamg_create(const pamg_params *p, pamg_handle **out) {
    if (!p || !out) return PAMG_ERR_ARG;
    *out = nullptr;
    if (p->multi_levels < 1 || p->multi_levels > p->n_split || p->n_split > kMaxLevels || p->n_split < 1 ||
        p->n_smooth < 0 || p->n_coarse < 0 || (p->solver < 1 || p->solver > 3) || !(p->dt > 0) ||
        p->theta != 1.0 || (p->halo_mode != 0 && p->halo_mode != 1) ||
        (p->coarse_solver != 0 && p->coarse_solver != 1) || p->fused < 0 || p->fused > 3 ||
        (p->arith != 0 && p->arith != 1) || (p->halo_exchange != 0 && p->halo_exchange != 1) ||
        (p->cycle != 0 && p->cycle != 1) || (p->cycle == 1 && p->solver == 2) || (p->op != 0 && p->op != 1) ||
        (p->op == 1 && (p->solver == 2 || p->coarse_solver == 1)))
        return PAMG_ERR_ARG;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return PAMG_ERR_NODEV;
    if (p->device < 0 || p->device >= ndev) return PAMG_ERR_NODEV;
    auto *h = new pamg_handle;
    h->p = *p;
    h->device = p->device;
    // PAMG_STREAM_CU_MASK=<n> | half (tests): the handle's stream runs on the first n CUs only (hipExtStreamCreateWithCUMask)
    // -- a persistent chain grid sized for every CU is then not co-resident (the chain's fail-safe path)
    const char *cm = getenv("PAMG_STREAM_CU_MASK");
    int ncu_mask = cm ? atoi(cm) : 0;
    if (cm && std::strcmp(cm, "half") == 0) {
        int n = 0;
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, p->device) != hipSuccess) n = 0;
        ncu_mask = n / 2;
    }
    auto make_stream = [&](hipStream_t *st) -> bool {
        if (ncu_mask <= 0) return hipStreamCreateWithFlags(st, hipStreamNonBlocking) == hipSuccess;
        std::vector<uint32_t> mask((size_t)(ncu_mask + 31) / 32, 0u);
        for (int c = 0; c < ncu_mask; ++c) mask[c / 32] |= 1u << (c % 32);
        return hipExtStreamCreateWithCUMask(st, (uint32_t)mask.size(), mask.data()) == hipSuccess;
    };
    if (hipSetDevice(h->device) != hipSuccess || !make_stream(&h->stream) ||
        hipStreamCreateWithFlags(&h->stream_comm, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&h->ev_packed, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&h->ev_sent[0], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&h->ev_sent[1], hipEventDisableTiming) != hipSuccess ||
        hipStreamCreateWithFlags(&h->stream_c, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&h->ev_fine, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&h->ev_coarse, hipEventDisableTiming) != hipSuccess) {
        delete h;
        return PAMG_ERR_HIP;
    }
    *out = h;
    return PAMG_OK;
}

int pamg_comm_unique_id(char out[128]) {
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess) return PAMG_ERR_COMM;
    static_assert(sizeof(id) == 128, "ncclUniqueId size");
    std::memcpy(out, &id, 128);
    return PAMG_OK;
}

int pamg_comm_init(pamg_handle *h, int nranks, int rank, const char id[128], int U, const int *owner) {
    if (!h || nranks < 1 || rank < 0 || rank >= nranks || !owner || U < 1) return PAMG_ERR_ARG;
    if (h->mesh_ready) { h->err = "pamg_comm_init must precede pamg_upload_mesh"; return PAMG_ERR_STATE; }
    ncclComm_t nc = nullptr;
    if (nranks > 1 && id) {   // id == NULL: detached partition (pamg_halo_loopback exchanges)
        if (h->comm) { h->err = "communicator already bound"; return PAMG_ERR_STATE; }
        HIPCHK(h, hipSetDevice(h->device));
        ncclUniqueId uid;
        std::memcpy(&uid, id, 128);
        // the communicator, the rank and the owner map are bound to the handle only once RCCL has initialised
        // it (a failure -- a peer that never joins, nccl_init's bound -- leaves the handle as it was, so a retry
        // can bind again)
        CHK(nccl_init(h, &nc, nranks, uid, rank));
    }
    h->nranks = nranks;
    h->rank = rank;
    h->owner.assign(owner, owner + U);
    if (nc) {
        h->comm = new Comm;
        h->comm->nccl = nc;
    }
    return PAMG_OK;
}

int pamg_comm_init_self(pamg_handle *h, const char id[128], int U, const int *part) {
    if (!h || !id || !part || U < 1) return PAMG_ERR_ARG;
    if (h->mesh_ready) { h->err = "pamg_comm_init_self must precede pamg_upload_mesh"; return PAMG_ERR_STATE; }
    if (h->comm) { h->err = "communicator already bound"; return PAMG_ERR_STATE; }
    HIPCHK(h, hipSetDevice(h->device));
    ncclUniqueId uid;
    std::memcpy(&uid, id, 128);
    // the plan and the communicator are bound only once RCCL has initialised it: a failure leaves
    // the handle as it was (no half-bound communicator, no self-peer parts), so a retry can bind
    ncclComm_t nc = nullptr;
    CHK(nccl_init(h, &nc, 1, uid, 0));
    h->nranks = 1;
    h->rank = 0;
    h->owner.assign(U, 0);
    h->vpart.assign(part, part + U);
    h->comm = new Comm;
    h->comm->nccl = nc;
    return PAMG_OK;
}

int pamg_comm_local_group(pamg_handle *const *hs, int n) {
    if (!hs || n < 2) return PAMG_ERR_ARG;
    std::vector<int> seen(n, 0);
    for (int a = 0; a < n; ++a) {
        pamg_handle *h = hs[a];
        if (!h || !h->mesh_ready || h->nranks != n || h->comm || h->rank < 0 || h->rank >= n || seen[h->rank]++)
            return PAMG_ERR_ARG;
        if (h->owner != hs[0]->owner) { h->err = "local group: the partitions' owner maps differ"; return PAMG_ERR_ARG; }
    }
    // create every handle's events first; bind the group only when all of them exist, so a
    // failure leaves no handle half-bound (a retry then sees h->comm == nullptr)
    std::vector<hipEvent_t> evs((size_t)2 * n, nullptr);
    for (int a = 0; a < n; ++a) {
        if (hipSetDevice(hs[a]->device) != hipSuccess ||
            hipEventCreateWithFlags(&evs[2 * a], hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&evs[2 * a + 1], hipEventDisableTiming) != hipSuccess) {
            for (hipEvent_t e : evs)
                if (e) (void)hipEventDestroy(e);
            hs[a]->err = "local group: hipEventCreate failed";
            return PAMG_ERR_HIP;
        }
    }
    auto *G = new LocalGroup;
    G->n = n;
    G->ready.resize((size_t)n * n);
    G->done.resize((size_t)n * n);
    G->refs = n;
    for (int a = 0; a < n; ++a) {
        pamg_handle *h = hs[a];
        h->comm = new Comm;
        h->comm->local = G;
        h->comm->seq.assign(n, 0);
        h->comm->ev_ready = evs[2 * a];
        h->comm->ev_done = evs[2 * a + 1];
    }
    return PAMG_OK;
}

int pamg_comm_info(pamg_handle *h, int *version, char *lib_path, int len) {
    if (!h) return PAMG_ERR_ARG;
    if (version) {
        int v = 0;
        if (ncclGetVersion(&v) != ncclSuccess) return PAMG_ERR_COMM;
        *version = v;
    }
    if (lib_path && len > 0) {
        Dl_info di{};
        const char *p = dladdr((void *)&ncclGetVersion, &di) && di.dli_fname ? di.dli_fname : "";
        std::strncpy(lib_path, p, (size_t)len - 1);
        lib_path[len - 1] = 0;
    }
    return !h->comm ? 0 : h->comm->local ? 2 : 1;
}

int pamg_upload_mesh(pamg_handle *h, int U, const double *X, const int *region, const int *neig, const int *fneig,
                     const int *dir) {
    if (!h || U < 1 || !X || !region || !neig || !fneig || !dir) return PAMG_ERR_ARG;
    CHK(settle(h));
    HIPCHK(h, hipSetDevice(h->device));
    if (h->agg) {
        (void)pamg_destroy(h->agg);
        h->agg = nullptr;
    }
    free_levels(h);
    h->U_global = U;
    h->owned.clear();
    if (!h->owner.empty() && (int)h->owner.size() != U) {
        h->err = "owner map size differs from the uploaded mesh";
        return PAMG_ERR_ARG;
    }
    if (!h->owner.empty()) {
        for (int g = 0; g < U; ++g) {
            if (h->owner[g] < 0 || h->owner[g] >= h->nranks) { h->err = "owner out of range"; return PAMG_ERR_ARG; }
            if (h->owner[g] == h->rank) h->owned.push_back(g);
        }
    } else {
        for (int g = 0; g < U; ++g) h->owned.push_back(g);
    }
    h->U = (int)h->owned.size();
    h->Xo.resize(6 * h->owned.size());
    for (size_t q = 0; q < h->owned.size(); ++q)
        for (int c = 0; c < 6; ++c) h->Xo[6 * q + c] = X[6 * (size_t)h->owned[q] + c];
    h->neig_local.clear();
    if (h->p.op == 1) {   // the local neighbours: the chain's workgroup lists, the wavefront's ticket order
        std::vector<int> g2l(U, -1);
        for (size_t q = 0; q < h->owned.size(); ++q) g2l[h->owned[q]] = (int)q;
        h->neig_local.assign(3 * h->owned.size(), -1);
        for (size_t q = 0; q < h->owned.size(); ++q)
            for (int f = 0; f < 3; ++f) {
                const int n = neig[3 * (size_t)h->owned[q] + f];
                if (n >= 1 && n <= U) h->neig_local[3 * q + f] = g2l[n - 1];
            }
    }
    for (int g = 0; g < U; ++g)
        for (int f = 0; f < 3; ++f) {
            const int n = neig[3 * g + f];
            if (n < 0 || n > U || (n && (fneig[3 * g + f] < 1 || fneig[3 * g + f] > 3))) {
                h->err = "inconsistent neighbour table at un_ele " + std::to_string(g + 1);
                return PAMG_ERR_ARG;
            }
        }
    const int S = h->p.n_split, Lc = h->p.multi_levels, Ul = h->U;
    h->slots = (1 << S) * 3;
    CHK(dev_alloc(h, &h->tov, (size_t)h->slots * 3 * std::max(Ul, 1)));
    CHK(dev_alloc(h, &h->tovo, (size_t)h->slots * 3 * std::max(Ul, 1)));
    HIPCHK(h, hipMemsetAsync(h->tov, 0, (size_t)h->slots * 3 * std::max(Ul, 1) * sizeof(double), h->stream));
    HIPCHK(h, hipMemsetAsync(h->tovo, 0, (size_t)h->slots * 3 * std::max(Ul, 1) * sizeof(double), h->stream));
    // level-1 geometry for the source term
    {
        std::vector<double> geo((size_t)std::max(Ul, 1) * kGeoStride, 0.0);
        const double pw = (double)(1 << S);
        for (int q = 0; q < Ul; ++q) {
            const double *x = X + 6 * (size_t)h->owned[q];
            double *g = &geo[(size_t)q * kGeoStride];
            g[0] = x[4]; g[1] = x[5];
            g[2] = (x[0] - x[4]) / pw; g[3] = (x[1] - x[5]) / pw;
            g[4] = (x[2] - x[4]) / pw; g[5] = (x[3] - x[5]) / pw;
        }
        CHK(dev_upload(h, &h->geo1, geo));
    }
    std::vector<int> pos[kMaxLevels + 1];   // hierarchical storage order of every level (Level::pos)
    hier_positions(S, Lc, pos);
    for (int l = 1; l <= Lc; ++l) {
        std::vector<char> seen(pos[l].size(), 0);
        for (int v : pos[l])
            if (v < 0 || v >= (int)pos[l].size() || seen[v]++) { h->err = "storage order is not a permutation"; return PAMG_ERR_STATE; }
    }
    for (int l = 1; l <= Lc; ++l) {
        if (h->coarse_only && l < Lc) continue;   // a replica of the coarsest level (agg_create)
        Level &L = h->lv[l];
        L.pos = pos[l];
        L.isplit = S - l + 1;
        // the contracted arithmetic is for solvers 1 and 3; Richardson's residual keeps the
        // reference's order (as the oracle's get_residual)
        L.arith = h->p.solver == 2 ? 0 : h->p.arith;
        L.richardson = h->p.solver == 2;
        L.nsub = 1 << (2 * L.isplit);
        L.N = (int64_t)L.nsub * Ul;
        // (a gap between the planes, so that a sub-element's three are not a power-of-two distance apart, measured
        // within noise: profiles/r05_e_asm_layouts.txt)
        L.pitch = std::max<int64_t>(64, (L.N + 63) / 64 * 64);
        double *base = nullptr;
        // level 1: the source term s' (SRC); level 2: RHSN_alt for the concurrent fused cycle and the face cycle's
        // level-1 restrictor fold, levels 3 .. L: RHSN_alt for the face cycle's folds of the coarser levels
        const size_t planes = 21;
        CHK(dev_alloc(h, &base, planes * (size_t)L.pitch));
        HIPCHK(h, hipMemsetAsync(base, 0, planes * (size_t)L.pitch * sizeof(double), h->stream));
        L.T = base; L.TNN = base + 3 * L.pitch; L.RHS = base + 6 * L.pitch; L.RES = base + 9 * L.pitch;
        L.TOLD = base + 12 * L.pitch;
        L.RHSN = base + 15 * L.pitch;   // restriction of the zero residual: valid
        L.RHSN_alt = (l >= 2) ? base + 18 * L.pitch : nullptr;
        L.SRC = (l == 1) ? base + 18 * L.pitch : nullptr;
        std::vector<double> stc((size_t)std::max(Ul, 1) * kStcStride, 0.0);
        for (int q = 0; q < Ul; ++q) {
            level_stencil(X + 6 * (size_t)h->owned[q], L.isplit, h->p.k, h->p.dt, h->p.omega,
                          &stc[(size_t)q * kStcStride]);
            if (!mass_is_p1_midpoint(&stc[(size_t)q * kStcStride])) {
                h->err = "mass matrix of un_ele " + std::to_string(h->owned[q] + 1) + " is not c*[[2,1,1],[1,2,1],[1,1,2]]";
                return PAMG_ERR_STATE;
            }
        }
        CHK(dev_upload(h, &L.stc, stc));
        std::vector<int2> sub(L.nsub);
        for (int e = 1; e <= L.nsub; ++e) {
            int irow, ipos, o;
            get_str_info(L.isplit, e, &irow, &ipos, &o);
            sub[L.pos[e - 1]] = make_int2(irow, ipos);
        }
        CHK(dev_upload(h, &L.subinfo, sub));
        CHK(dev_upload(h, &L.d_pos, L.pos));
        if (l == 1) HIPCHK(h, launch_source(h->stream, L, h->geo1, h->p.k));   // s' of get_RHS, once
        CHK(build_halo(h, l, X, neig, fneig, dir));
        if (h->p.op == 1) {
            std::vector<int4> fnb;
            std::vector<double> fface;
            std::vector<int> fsx;
            CHK(build_face(h, l, X, neig, fneig, dir, fnb, fface, fsx));
            CHK(dev_upload(h, &L.fnb, fnb));
            CHK(dev_upload(h, &L.fface, fface));
            CHK(dev_upload(h, &L.fsx, fsx));
            // the up positions without halo words, the up ones with words, then the down ones (the
            // order inside a colour is free: a colour pass reads only the other colour)
            auto has_words = [&](int j) {
                if (j >= (int)L.halo.hsub.size()) return false;
                const int4 e = L.halo.hsub[j];
                return (e.x | e.y | e.z) != 0;
            };
            std::vector<int> cpos;
            L.nui = 0;
            for (int pass = 0; pass < 3; ++pass)
                for (int j = 0; j < L.nsub; ++j) {
                    const bool up = fnb[j].w != 0;
                    if (pass == 0 ? up && !has_words(j) : pass == 1 ? up && has_words(j) : !up) cpos.push_back(j);
                    if (pass == 0 && up && !has_words(j)) ++L.nui;
                }
            L.nup = 0;
            for (int j = 0; j < L.nsub; ++j) L.nup += fnb[j].w != 0;
            L.ndn = L.nsub - L.nup;
            L.words_up = true;
            for (int j = 0; j < L.nsub && j < (int)L.halo.hsub.size(); ++j) {
                const int4 e = L.halo.hsub[j];
                if ((e.x | e.y | e.z) && !fnb[j].w) L.words_up = false;
            }
            CHK(dev_upload(h, &L.cpos, cpos));
            std::vector<int4> cnb(cpos.size());
            for (size_t i = 0; i < cpos.size(); ++i) cnb[i] = fnb[cpos[i]];
            CHK(dev_upload(h, &L.cnb, cnb));
            // the two-sweep passes' gather table (k_face_pp, Level::gtab): for every halo slot of every local
            // un_ele, the neighbour's boundary sub-element e whose words fill it (hface: this un_ele's words
            // into the neighbour; the neighbour's record back: its words into this one, reversed or not) and,
            // for each face of e, where the value across it lives
            if (face_tile_shape(L)) {
                const int m = 1 << L.isplit, sl = h->slots, ns = L.nsub;
                std::vector<int4> gf((size_t)std::max(Ul, 1) * 3, make_int4(-1, 0, 0, 0));   // {v, fv, rev v->u, rev u->v}
                for (int q = 0; q < Ul; ++q)
                    for (int f = 1; f <= 3; ++f) {
                        const int4 r = L.halo.hface[3 * (size_t)q + f - 1];
                        const int mode = r.x & 3;
                        if (mode == 0) continue;
                        if (mode == 2) { gf[3 * (size_t)q + f - 1] = make_int4(-2, 0, 0, 0); continue; }
                        const int v = r.y / (3 * sl), fv = (r.y - v * 3 * sl) / sl + 1;
                        const int4 rv = L.halo.hface[3 * (size_t)v + fv - 1];
                        if ((rv.x & 3) != 1 || rv.y != q * 3 * sl + (f - 1) * sl) {
                            h->err = "face operator: asymmetric halo records between un_eles " + std::to_string(q) + " and " + std::to_string(v);
                            return PAMG_ERR_STATE;
                        }
                        gf[3 * (size_t)q + f - 1] = make_int4(v, fv, rv.x >> 2, r.x >> 2);
                    }
                std::vector<int> E(3 * (size_t)m, -1);   // boundary sub-element at position i of face f
                for (int j = 0; j < ns && j < (int)L.halo.hsub.size(); ++j) {
                    const int4 e = L.halo.hsub[j];
                    if (e.x) E[e.x - 1] = j;
                    if (e.y) E[m + e.y - 1] = j;
                    if (e.z) E[2 * m + e.z - 1] = j;
                }
                for (int v : E)
                    if (v < 0) { h->err = "face operator: a face position without its boundary sub-element"; return PAMG_ERR_STATE; }
                static const int fmface[3] = {1, 3, 2};   // un_ele face under sub-element face fi (pamg_face.hip cFMface)
                std::vector<int4> gt((size_t)std::max(Ul, 1) * 3 * m, make_int4(-1, 0, 0, 0));
                std::vector<int> gp(gt.size(), 0);
                for (int q = 0; q < Ul; ++q)
                    for (int f = 1; f <= 3; ++f) {
                        const int4 g = gf[3 * (size_t)q + f - 1];
                        for (int sp = 1; sp <= m; ++sp) {
                            int4 &o = gt[(3 * (size_t)q + f - 1) * m + sp - 1];
                            if (g.x < 0) { o = make_int4(g.x, 0, 0, 0); continue; }
                            const int e = E[(g.y - 1) * m + (g.z ? m - sp + 1 : sp) - 1];
                            const int4 nb = fnb[e];
                            const int nbf[3] = {nb.x, nb.y, nb.z};
                            int y[3];
                            for (int fi = 0; fi < 3; ++fi) {
                                if (nbf[fi] >= 0) { y[fi] = g.x * ns + nbf[fi]; continue; }
                                const int mf = fmface[fi], spp = -nbf[fi];
                                if (mf == g.y) {   // across to this un_ele: its own boundary sub-element
                                    y[fi] = -1 - E[(f - 1) * m + (g.w ? m - spp + 1 : spp) - 1];
                                    continue;
                                }
                                const int4 g2 = gf[3 * (size_t)g.x + mf - 1];   // a corner: the neighbour's other face
                                if (g2.x >= 0) y[fi] = g2.x * ns + E[(g2.y - 1) * m + (g2.z ? m - spp + 1 : spp) - 1];
                                else if (g2.x == -1)
                                    y[fi] = -(1 + ns + 3 * (L.halo.hface[3 * (size_t)g.x + mf - 1].z + spp - 1) + mf - 1);
                                else y[fi] = -1 - e;   // another rank: k_face_pp is single-domain (never read)
                            }
                            o = make_int4(g.x * ns + e, y[0], y[1], y[2]);
                            gp[(3 * (size_t)q + f - 1) * m + sp - 1] = (nb.x >= 0) | ((nb.y >= 0) << 1) | ((nb.z >= 0) << 2);
                        }
                    }
                CHK(dev_upload(h, &L.gtab, gt));
                CHK(dev_upload(h, &L.gpat, gp));
            }
        }
        HaloPlan &P = L.halo;
        CHK(dev_upload(h, &P.d_local, P.local));
        CHK(dev_upload(h, &P.d_bc, P.bc));
        CHK(dev_upload(h, &P.d_remote, P.remote));
        CHK(dev_upload(h, &P.d_recv_dst, P.recv_dst));
        CHK(dev_upload(h, &P.d_hface, P.hface));
        CHK(dev_upload(h, &P.d_hsub, P.hsub));
        {
            std::vector<int> bpos;
            for (int q = 0; q < (int)P.hsub.size(); ++q)
                if (P.hsub[q].x | P.hsub[q].y | P.hsub[q].z) bpos.push_back(q);
            P.nbpos = (int)bpos.size();
            if (bpos.empty()) bpos.push_back(0);
            CHK(dev_upload(h, &P.d_bpos, bpos));
        }
        CHK(dev_upload(h, &P.d_bcv, P.bcv));
        CHK(dev_upload(h, &P.d_surf, P.surf));
        CHK(dev_alloc(h, &P.d_told_halo, 3 * (size_t)P.n_told));
        CHK(refresh_told_halo(h, l));
        CHK(dev_alloc(h, &P.d_send, 6 * P.remote.size()));
        if (l == 1 && !P.remote.empty()) CHK(dev_alloc(h, &P.d_send_b, 6 * P.remote.size()));
        CHK(dev_alloc(h, &P.d_recv, 6 * P.recv_dst.size()));
    }
    // initial condition (:237-252): tnew = 0, region 4 => 1 on level 1
    if (!h->coarse_only) {
        Level &L1 = h->lv[1];
        bool any = false;
        for (int q = 0; q < Ul; ++q) any |= region[h->owned[q]] == 4;
        if (any) {
            std::vector<double> t(3 * (size_t)L1.pitch, 0.0);
            for (int q = 0; q < Ul; ++q)
                if (region[h->owned[q]] == 4)
                    for (int c = 0; c < 3; ++c)
                        for (int e = 0; e < L1.nsub; ++e) t[c * L1.pitch + (size_t)q * L1.nsub + e] = 1.0;
            // behind the memset of the level's planes on the same stream
            HIPCHK(h, hipMemcpyAsync(L1.T, t.data(), t.size() * sizeof(double), hipMemcpyHostToDevice, h->stream));
            HIPCHK(h, hipStreamSynchronize(h->stream));
        }
        HIPCHK(h, launch_copy(h->stream, L1.T, L1.TNN, 3 * L1.pitch));
        h->tnn_level = 1;
    }
    HIPCHK(h, hipStreamSynchronize(h->stream));
    h->mesh_ready = true;
    return agg_create(h, U, X, region, neig, fneig, dir);
}

int pamg_owned_count(pamg_handle *h) { return h ? h->U : PAMG_ERR_ARG; }

int pamg_nsub(pamg_handle *h, int level) {
    if (!h) return PAMG_ERR_ARG;
    CHK(check_level(h, level));
    return h->lv[level].nsub;
}

int pamg_tnn_level(pamg_handle *h) { return h ? h->tnn_level : PAMG_ERR_ARG; }

int pamg_set_state(pamg_handle *h, int level, int what, const double *host) {
    if (!h || !host) return PAMG_ERR_ARG;
    CHK(settle(h));
    if (what == PAMG_TNEW_NONLIN) { CHK(check_level(h, level)); h->tnn_level = level; }
    CHK(check_level(h, level));
    Level &L = h->lv[level];
    double *dst = what == PAMG_SOURCE ? nullptr : field_ptr(h, level, what);   // the source is read-only
    if (!dst) return PAMG_ERR_ARG;
    CHK(ensure_scratch(h, 3 * (size_t)L.N * sizeof(double)));
    HIPCHK(h, hipMemcpyAsync(h->scratch, host, 3 * (size_t)L.N * sizeof(double), hipMemcpyHostToDevice, h->stream));
    HIPCHK(h, launch_to_soa(h->stream, L, h->scratch, dst));
    if (what == PAMG_TOLD) CHK(refresh_told_halo(h, level));
    if (what == PAMG_RESIDUAL) h->rhsn_valid = false;
    CHK(sync_stream(h, h->stream));
    return PAMG_OK;
}

int pamg_get_state(pamg_handle *h, int level, int what, double *host) {
    if (!h || !host) return PAMG_ERR_ARG;
    CHK(settle(h));
    if (what == PAMG_TNEW_NONLIN) level = h->tnn_level;
    CHK(check_level(h, level));
    Level &L = h->lv[level];
    double *src = field_ptr(h, level, what);
    if (!src) return PAMG_ERR_ARG;
    CHK(ensure_scratch(h, 3 * (size_t)L.N * sizeof(double)));
    HIPCHK(h, launch_to_aos(h->stream, L, src, h->scratch));
    HIPCHK(h, hipMemcpyAsync(host, h->scratch, 3 * (size_t)L.N * sizeof(double), hipMemcpyDeviceToHost, h->stream));
    CHK(sync_stream(h, h->stream));
    return PAMG_OK;
}

int pamg_get_overlap(pamg_handle *h, double *tov, double *tovo) {
    if (!h || !h->mesh_ready) return PAMG_ERR_STATE;
    CHK(settle(h));
    const size_t n = (size_t)h->slots * 3 * h->U * sizeof(double);
    if (tov) HIPCHK(h, hipMemcpyAsync(tov, h->tov, n, hipMemcpyDeviceToHost, h->stream));
    if (tovo) HIPCHK(h, hipMemcpyAsync(tovo, h->tovo, n, hipMemcpyDeviceToHost, h->stream));
    CHK(sync_stream(h, h->stream));
    return PAMG_OK;
}

// tnn_dead: the caller runs a V-cycle next, whose first smoother call rewrites tnew_nonlin
// (:327) before any read, so the :317 copy is not stored (pamg_run); told_lazy: that V-cycle
// is the fused one, whose k_overlap_static refreshes the compact told copy of the halo from
// TOLD itself (one launch instead of k_told_halo + k_overlap_static)
int begin_timestep(pamg_handle *h, bool tnn_dead, bool told_lazy = false, bool defer_rhs = false) {
    CHK(check_level(h, 1));
    // the first launch of the step's fused V-cycle does k_rhs's work (Richardson: the resident
    // launch, which also rebuilds the RHS where get_residual does)
    if (defer_rhs && (h->p.solver != 2 || fused_ok(h))) {
        h->tnn_level = 1;
        h->overlap_static_l1 = false;
        h->told_halo_stale_l1 = true;
        h->rhs_pending = true;
        return PAMG_OK;
    }
    h->tnn_level = 1;
    if (h->p.solver == 2) {   // solve_Richardson never calls get_RHS inside the smoother
        Level &L = h->lv[1];
        HIPCHK(h, launch_copy(h->stream, L.T, L.TOLD, 3 * L.pitch));
        HIPCHK(h, launch_copy(h->stream, L.T, L.TNN, 3 * L.pitch));
        return refresh_told_halo(h, 1);
    }
    CHK(rhs_level1(h, tnn_dead ? 2 : 1));   // also the compact told copy of the halo (refresh_told_halo)
    if (PAMG_RHS_TOLD_HALO || told_lazy) {
        h->overlap_static_l1 = false;
        h->told_halo_stale_l1 = !PAMG_RHS_TOLD_HALO;
        return PAMG_OK;
    }
    return refresh_told_halo(h, 1);
}

int pamg_begin_timestep(pamg_handle *h) {
    if (!h) return PAMG_ERR_ARG;
    CHK(settle(h));
    return begin_timestep(h, false);
}

int pamg_copy_to_nonlin(pamg_handle *h, int level) {
    if (!h) return PAMG_ERR_ARG;
    CHK(settle(h));
    CHK(check_level(h, level));
    Level &L = h->lv[level];
    HIPCHK(h, launch_copy(h->stream, L.T, L.TNN, 3 * L.pitch));
    h->tnn_level = level;
    return PAMG_OK;
}

int pamg_smoother(pamg_handle *h, int level, int n_calls) {
    if (!h || n_calls < 0) return PAMG_ERR_ARG;
    CHK(settle(h));
    CHK(check_level(h, level));
    if (h->tnn_level != level) {
        h->err = "smoother: tnew_nonlin holds another level (call pamg_copy_to_nonlin first)";
        return PAMG_ERR_STATE;
    }
    CHK(smooth(h, level, false, h->p.n_smooth * n_calls));
    return h->p.op == 1 ? face_chain_check(h) : PAMG_OK;
}

int pamg_sweep(pamg_handle *h, int level, int n_sweeps) {
    if (!h || n_sweeps < 0) return PAMG_ERR_ARG;
    CHK(settle(h));
    CHK(check_level(h, level));
    if (h->tnn_level != level) {
        h->err = "sweep: tnew_nonlin holds another level (call pamg_copy_to_nonlin first)";
        return PAMG_ERR_STATE;
    }
    CHK(smooth(h, level, false, n_sweeps));
    return h->p.op == 1 ? face_chain_check(h) : PAMG_OK;
}

int pamg_restrictor(pamg_handle *h, int level) {
    if (!h) return PAMG_ERR_ARG;
    CHK(settle(h));
    CHK(check_level(h, level));
    return restrict_(h, level);
}

int pamg_get_residual(pamg_handle *h, int level) {
    if (!h) return PAMG_ERR_ARG;
    CHK(settle(h));
    CHK(check_level(h, level));
    return residual(h, level);
}

int pamg_prolongator(pamg_handle *h, int level) {
    if (!h) return PAMG_ERR_ARG;
    CHK(settle(h));
    CHK(check_level(h, level));
    return prolong(h, level, false);
}

int vcycle(pamg_handle *h, int n, bool dead_after) {
    CHK(check_level(h, 1));
    // the fused op = 0 forms wait only for the exchange that read the send buffer they pack; the others may
    // touch anything an early exchange still in flight touches
    if (!(h->p.cycle == 0 && fused_ok(h))) CHK(settle(h));
    if (h->p.cycle == 1) {
        if (corrected_resident_ok(h)) return vcycle_corrected_resident(h, n);
        if (face_corrected_pp_ok(h)) return vcycle_corrected_face_pp(h, n);
        for (int c = 0; c < n; ++c) CHK(vcycle_corrected(h));
        return h->p.op == 1 ? face_chain_check(h) : PAMG_OK;
    }
    if (fused_ok(h)) return vcycle_fused(h, n, dead_after);
    if (face_cycle_fusable(h)) return vcycle_face_fused(h, n);
    for (int c = 0; c < n; ++c) CHK(vcycle_steps(h));
    return h->p.op == 1 ? face_chain_check(h) : PAMG_OK;
}

int pamg_vcycle(pamg_handle *h, int n) {
    if (!h || n < 0) return PAMG_ERR_ARG;
    CHK(vcycle(h, n, false));
    return comm_error(h);
}

int pamg_direct_solve(pamg_handle *h, int level) {
    if (!h) return PAMG_ERR_ARG;
    CHK(settle(h));
    CHK(check_level(h, level));
    return direct_solve(h, level);
}

int pamg_block_inverse(pamg_handle *h, int n, long nb, const double *A, double *inv, int *errorflag) {
    if (!h || n < 1 || n > 8 || nb < 0 || (nb > 0 && (!A || !inv || !errorflag))) return PAMG_ERR_ARG;
    if (nb == 0) return PAMG_OK;
    HIPCHK(h, hipSetDevice(h->device));
    const size_t nd = (size_t)n * n * (size_t)nb;
    double *dA = nullptr, *dI = nullptr;
    int *dE = nullptr;
    int rc = PAMG_OK;
    if (hipMalloc((void **)&dA, nd * sizeof(double)) != hipSuccess ||
        hipMalloc((void **)&dI, nd * sizeof(double)) != hipSuccess ||
        hipMalloc((void **)&dE, (size_t)nb * sizeof(int)) != hipSuccess ||
        hipMemcpyAsync(dA, A, nd * sizeof(double), hipMemcpyHostToDevice, h->stream) != hipSuccess ||
        launch_block_inverse(h->stream, n, nb, dA, dI, dE) != hipSuccess ||
        hipMemcpyAsync(inv, dI, nd * sizeof(double), hipMemcpyDeviceToHost, h->stream) != hipSuccess ||
        hipMemcpyAsync(errorflag, dE, (size_t)nb * sizeof(int), hipMemcpyDeviceToHost, h->stream) != hipSuccess ||
        hipStreamSynchronize(h->stream) != hipSuccess) {
        h->err = "pamg_block_inverse: HIP error";
        rc = PAMG_ERR_HIP;
    }
    (void)hipFree(dA);
    (void)hipFree(dI);
    (void)hipFree(dE);
    return rc;
}

int pamg_run(pamg_handle *h, int ntime, int n_multigrid) {
    if (!h || ntime < 0 || n_multigrid < 0) return PAMG_ERR_ARG;
    CHK(settle(h));
    {
        // the resident schedule runs the whole loop as one launch: a step touches only its own
        // tiles (told := tnew, the RHS from it and s', n_multigrid cycles), so every tile goes
        // through all ntime steps on-chip and only the run's final state is stored
        const int L = h->p.multi_levels;
        if (ntime >= 2 && n_multigrid >= 1 && h->p.cycle == 0 && h->p.fused == 3 && h->p.coarse_solver == 0 &&
            h->p.op == 0 && h->p.halo_exchange == 0 && !h->coarse_ahead && call_schedule(h) == 3 && fused_ok(h) &&
            vcycle_resident_run_supported(h->p.n_split, L) && vcycle_rhsf_supported(h->p.n_split) &&
            !PAMG_RHS_TOLD_HALO) {
            int rc = begin_timestep(h, true, true, true);
            if (rc == PAMG_OK) rc = vcycle_fused(h, n_multigrid, false, ntime);
            if (rc != PAMG_OK) {
                h->coarse_ahead = false;
                h->rhs_pending = false;
                return rc;
            }
            return comm_error(h);
        }
    }
    for (int t = 0; t < ntime; ++t) {
        const int L = h->p.multi_levels;
        const bool fused_next = n_multigrid > 0 && fused_ok(h);
        // told := tnew and the RHS inside the step's first level-1 launch when that launch is a
        // pipelined one on the one-stream schedule
        // (the resident schedule starts the step in its one launch, for any n_multigrid)
        const int cs = call_schedule(h);
        const bool defer_rhs = fused_next && h->p.fused == 3 && L > 1 && h->p.halo_exchange == 0 &&
                               vcycle_rhsf_supported(h->p.n_split) &&
                               (cs == 3 ? vcycle_resident_supported(h->p.n_split, L)
                                        : cs == 1 && (n_multigrid > 1 || t + 1 < ntime)) &&
                               !PAMG_RHS_TOLD_HALO;
        int rc = begin_timestep(h, n_multigrid > 0 && h->p.cycle == 0, fused_next, defer_rhs);
        if (rc == PAMG_OK) rc = vcycle(h, n_multigrid, t + 1 < ntime);   // a step's leftovers die in the next one
        if (rc != PAMG_OK) {
            h->coarse_ahead = false;
            h->rhs_pending = false;
            return rc;
        }
    }
    return comm_error(h);
}

int pamg_synchronize(pamg_handle *h) {
    if (!h) return PAMG_ERR_ARG;
    CHK(sync_stream(h, h->stream));
    if (h->sent_pending[0] || h->sent_pending[1]) CHK(sync_stream(h, h->stream_comm));
    return PAMG_OK;
}

int pamg_timing_enable(pamg_handle *h, unsigned mask) {
    if (!h) return PAMG_ERR_ARG;
    h->timing.mask = mask;
    return PAMG_OK;
}

int pamg_early_exchange_times(pamg_handle *h, double t[3]) {
    if (!h || !t) return PAMG_ERR_ARG;
    if (!h->xe_ev_valid) return PAMG_ERR_STATE;
    CHK(sync_stream(h, h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream_comm));
    for (int k = 0; k < 3; ++k) {
        float ms = 0.f;
        HIPCHK(h, hipEventElapsedTime(&ms, h->xe_ev[0], h->xe_ev[k + 1]));
        t[k] = 1e3 * (double)ms;
    }
    return PAMG_OK;
}

int pamg_timing_reset(pamg_handle *h) {
    if (!h) return PAMG_ERR_ARG;
    h->xe_ev_valid = false;
    CHK(drain_timing(h));
    for (int k = 0; k < PAMG_K_COUNT; ++k) {
        h->timing.ms[k] = 0; h->timing.count[k] = 0; h->timing.bytes[k] = 0; h->timing.seq[k] = 0;
    }
    return PAMG_OK;
}

int pamg_vcycle_flops(pamg_handle *h, double *flops_per_cycle) {
    if (!h || !flops_per_cycle) return PAMG_ERR_ARG;
    if (!h->mesh_ready) return PAMG_ERR_STATE;
    *flops_per_cycle = vcycle_flops(h);
    return PAMG_OK;
}

int pamg_set_call_schedule(pamg_handle *h, int schedule) {
    if (!h || schedule < 0 || schedule > 3) return PAMG_ERR_ARG;
    h->call_schedule = schedule;
    return PAMG_OK;
}

int pamg_timing_stride(pamg_handle *h, int every) {
    if (!h || every < 1) return PAMG_ERR_ARG;
    h->timing.stride = every;
    return PAMG_OK;
}

int pamg_timing_read(pamg_handle *h, int kid, double *ms_total, long *launches, double *bytes_total) {
    if (!h || kid < 0 || kid >= PAMG_K_COUNT) return PAMG_ERR_ARG;
    CHK(drain_timing(h));
    if (ms_total) *ms_total = h->timing.ms[kid];
    if (launches) *launches = h->timing.count[kid];
    if (bytes_total) *bytes_total = h->timing.bytes[kid];
    return PAMG_OK;
}

int pamg_timing_issued(pamg_handle *h, int kid, long *issued) {
    if (!h || !issued || kid < 0 || kid >= PAMG_K_COUNT) return PAMG_ERR_ARG;
    *issued = h->timing.seq[kid];
    return PAMG_OK;
}

int pamg_sweep_bench(pamg_handle *h, int sweeps, int assembled, double *ms_avg, double *bytes_per_launch) {
    if (!h || sweeps < 1) return PAMG_ERR_ARG;
    CHK(settle(h));
    CHK(check_level(h, 1));
    Level &L = h->lv[1];
    const double rdt = 1 / h->p.dt;
    CHK(ensure_scratch(h, 3 * (size_t)L.pitch * sizeof(double)));
    if (assembled && !L.blocks) {
        CHK(dev_alloc(h, &L.blocks, asm_blocks_doubles(L)));
        HIPCHK(h, launch_build_blocks(h->stream, L, rdt));
    }
    const double bytes = assembled ? 168.0 * (double)L.N : 72.0 * (double)L.N + 168.0 * h->U;
    const unsigned saved = h->timing.mask;
    CHK(drain_timing(h));
    const double ms0 = h->timing.ms[PAMG_K_SWEEP_BENCH];
    const long n0 = h->timing.count[PAMG_K_SWEEP_BENCH];
    h->timing.mask |= 1u << PAMG_K_SWEEP_BENCH;
    for (int s = 0; s < sweeps; ++s) {
        Span sp(h, PAMG_K_SWEEP_BENCH, bytes);
        if (assembled) HIPCHK(h, launch_sweep_assembled(h->stream, L, h->scratch, rdt));
        else HIPCHK(h, launch_sweep_stencil(h->stream, L, h->scratch, rdt));
    }
    h->timing.mask = saved;
    CHK(drain_timing(h));
    const long n = h->timing.count[PAMG_K_SWEEP_BENCH] - n0;
    if (ms_avg) *ms_avg = (h->timing.ms[PAMG_K_SWEEP_BENCH] - ms0) / std::max(1L, n);
    if (bytes_per_launch) *bytes_per_launch = bytes;
    return PAMG_OK;
}

int pamg_sweep_bench_output(pamg_handle *h, int assembled, double *host) {
    if (!h || !host) return PAMG_ERR_ARG;
    CHK(settle(h));
    CHK(check_level(h, 1));
    Level &L = h->lv[1];
    const double rdt = 1 / h->p.dt;
    // the sweep's output planes, then its (3, nsub, U) image
    CHK(ensure_scratch(h, 6 * (size_t)L.pitch * sizeof(double)));
    if (assembled && !L.blocks) {
        CHK(dev_alloc(h, &L.blocks, asm_blocks_doubles(L)));
        HIPCHK(h, launch_build_blocks(h->stream, L, rdt));
    }
    if (assembled) HIPCHK(h, launch_sweep_assembled(h->stream, L, h->scratch, rdt));
    else HIPCHK(h, launch_sweep_stencil(h->stream, L, h->scratch, rdt));
    double *img = h->scratch + 3 * L.pitch;
    HIPCHK(h, launch_to_aos(h->stream, L, h->scratch, img));
    HIPCHK(h, hipMemcpyAsync(host, img, 3 * (size_t)L.N * sizeof(double), hipMemcpyDeviceToHost, h->stream));
    CHK(sync_stream(h, h->stream));
    return PAMG_OK;
}

int pamg_last_error(pamg_handle *h, char *buf, int len) {
    if (!h || !buf || len <= 0) return PAMG_ERR_ARG;
    std::strncpy(buf, h->err.c_str(), (size_t)len - 1);
    buf[len - 1] = 0;
    return PAMG_OK;
}

int pamg_destroy(pamg_handle *h) {
    if (!h) return PAMG_OK;
    (void)hipSetDevice(h->device);
    (void)face_gates_drain(h);
    if (h->agg) {
        (void)pamg_destroy(h->agg);
        h->agg = nullptr;
    }
    (void)hipStreamSynchronize(h->stream);
    if (h->stream_fb) (void)hipStreamSynchronize(h->stream_fb);
    (void)hipStreamSynchronize(h->stream_comm);
    if (h->stream_c) (void)hipStreamSynchronize(h->stream_c);
    free_levels(h);
    dev_free(h->scratch);
    dev_free(h->chain_tmo);
    if (h->gate) (void)hipFree(h->gate);
    if (h->gate_stat) (void)hipHostFree(h->gate_stat);
    if (h->stream_fb) (void)hipStreamDestroy(h->stream_fb);
    dev_free(h->xc_done);
    dev_free(h->xe_done);
    for (auto e : h->xe_ev)
        if (e) (void)hipEventDestroy(e);
    if (h->xc_sig) (void)hipFree(h->xc_sig);
    for (auto e : h->timing.pool) (void)hipEventDestroy(e);
    for (auto &r : h->timing.pending) { (void)hipEventDestroy(r.a); (void)hipEventDestroy(r.b); }
    if (h->borrowed_stream) {   // a coarsest-level replica: the streams are its parent's
        delete h;
        return PAMG_OK;
    }
    if (h->comm) {
        if (h->comm->nccl) nccl_release(h->comm->nccl);
        if (h->comm->ev_ready) (void)hipEventDestroy(h->comm->ev_ready);
        if (h->comm->ev_done) (void)hipEventDestroy(h->comm->ev_done);
        if (LocalGroup *G = h->comm->local) {
            bool last;
            {
                std::lock_guard<std::mutex> lk(G->mu);
                last = --G->refs == 0;
            }
            if (last) delete G;
        }
        delete h->comm;
    }
    (void)hipStreamSynchronize(h->stream_comm);
    if (h->stream_c) (void)hipStreamSynchronize(h->stream_c);
    for (hipEvent_t e : {h->ev_packed, h->ev_sent[0], h->ev_sent[1], h->ev_fine, h->ev_coarse})
        if (e) (void)hipEventDestroy(e);
    (void)hipStreamDestroy(h->stream_comm);
    if (h->stream_c) (void)hipStreamDestroy(h->stream_c);
    if (!h->borrowed_stream) (void)hipStreamDestroy(h->stream);
    delete h;
    return PAMG_OK;
}

}  // extern "C"
