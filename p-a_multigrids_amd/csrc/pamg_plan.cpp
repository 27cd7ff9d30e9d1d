// Host-only access to the halo plan of update_overlaps (splitting.F90:1210-1397)
// for a partitioned mesh, and the single-process loopback exchange used to test
// the partitioned device path on one GPU.
#include <cstring>
#include <vector>

#include "pamg_internal.h"

struct pamg_plan {
    std::vector<int> owned;
    pamg::HaloPlan P;
};

extern "C" {

int pamg_plan_build(int U, const double *X, const int *neig, const int *fneig, const int *dir, int n_split,
                    int level, int nranks, int rank, const int *owner, pamg_plan **out) {
    if (U < 1 || !X || !neig || !fneig || !dir || !out || n_split < 1 || n_split > pamg::kMaxLevels ||
        level < 1 || level > n_split || nranks < 1 || rank < 0 || rank >= nranks)
        return PAMG_ERR_ARG;
    pamg_handle h;   // host-side fields only, no device resources
    h.U_global = U;
    h.nranks = nranks;
    h.rank = rank;
    if (owner && nranks > 1) h.owner.assign(owner, owner + U);
    for (int g = 0; g < U; ++g)
        if (h.owner.empty() || h.owner[g] == rank) h.owned.push_back(g);
    h.U = (int)h.owned.size();
    h.slots = (1 << n_split) * 3;
    h.lv[level].isplit = n_split - level + 1;
    h.lv[level].nsub = 1 << (2 * h.lv[level].isplit);
    int rc = pamg::build_halo(&h, level, X, neig, fneig, dir);
    if (rc != PAMG_OK) return rc;
    auto *p = new pamg_plan;
    p->owned = h.owned;
    p->P = h.lv[level].halo;
    *out = p;
    return PAMG_OK;
}

int pamg_plan_sizes(const pamg_plan *p, int *s) {
    if (!p || !s) return PAMG_ERR_ARG;
    s[0] = (int)p->owned.size();
    s[1] = (int)p->P.local.size();
    s[2] = (int)p->P.bc.size();
    s[3] = (int)p->P.remote.size();
    s[4] = (int)p->P.recv_dst.size();
    s[5] = (int)p->P.peers.size();
    return PAMG_OK;
}

int pamg_plan_get(const pamg_plan *p, int *owned, int *local_src, int *local_dst, int *bc_dst, double *bc_val,
                  int *remote_src, int *peers, int *send_off, int *recv_dst, int *recv_off) {
    if (!p) return PAMG_ERR_ARG;
    const pamg::HaloPlan &P = p->P;
    if (owned) std::memcpy(owned, p->owned.data(), sizeof(int) * p->owned.size());
    for (size_t i = 0; i < P.local.size(); ++i) {
        if (local_src) local_src[i] = P.local[i].src;
        if (local_dst) local_dst[i] = P.local[i].dst;
    }
    for (size_t i = 0; i < P.bc.size(); ++i) {
        if (bc_dst) { bc_dst[2 * i] = P.bc[i].dst_a; bc_dst[2 * i + 1] = P.bc[i].dst_b; }
        if (bc_val) { bc_val[2 * i] = P.bc[i].val_a; bc_val[2 * i + 1] = P.bc[i].val_b; }
    }
    for (size_t i = 0; i < P.remote.size(); ++i)
        if (remote_src) remote_src[i] = P.remote[i].src;
    if (peers) std::memcpy(peers, P.peers.data(), sizeof(int) * P.peers.size());
    if (send_off) {
        if (P.send_peer_off.empty()) send_off[0] = 0;
        else std::memcpy(send_off, P.send_peer_off.data(), sizeof(int) * P.send_peer_off.size());
    }
    if (recv_dst) std::memcpy(recv_dst, P.recv_dst.data(), sizeof(int) * P.recv_dst.size());
    if (recv_off) {
        if (P.recv_peer_off.empty()) recv_off[0] = 0;
        else std::memcpy(recv_off, P.recv_peer_off.data(), sizeof(int) * P.recv_peer_off.size());
    }
    return PAMG_OK;
}

void pamg_plan_free(pamg_plan *p) { delete p; }

int pamg_halo_loopback(pamg_handle *const *hs, int n, int level) {
    if (!hs || n < 1) return PAMG_ERR_ARG;
    for (int a = 0; a < n; ++a) {
        if (!hs[a] || !hs[a]->mesh_ready || level < 1 || level > hs[a]->p.multi_levels) return PAMG_ERR_ARG;
        if (hipStreamSynchronize(hs[a]->stream) != hipSuccess) return PAMG_ERR_HIP;
    }
    for (int b = 0; b < n; ++b) {           // receiver
        pamg_handle *hb = hs[b];
        const pamg::HaloPlan &Pb = hb->lv[level].halo;
        for (size_t qb = 0; qb < Pb.peers.size(); ++qb) {
            const int src_rank = Pb.peers[qb];
            pamg_handle *ha = nullptr;
            for (int a = 0; a < n; ++a)
                if (hs[a]->rank == src_rank) ha = hs[a];
            if (!ha) return PAMG_ERR_ARG;
            const pamg::HaloPlan &Pa = ha->lv[level].halo;
            int qa = -1;
            for (size_t q = 0; q < Pa.peers.size(); ++q)
                if (Pa.peers[q] == hb->rank) qa = (int)q;
            const size_t nr = (size_t)(Pb.recv_peer_off[qb + 1] - Pb.recv_peer_off[qb]);
            const size_t ns = qa < 0 ? 0 : (size_t)(Pa.send_peer_off[qa + 1] - Pa.send_peer_off[qa]);
            if (nr != ns) { hb->err = "loopback: send/recv counts differ"; return PAMG_ERR_STATE; }
            if (nr == 0) continue;
            // on the receiver's stream, so its unpack below is ordered behind the copy (a blocking
            // hipMemcpy runs on the null stream, which the non-blocking handle streams do not wait for)
            if (hipMemcpyAsync(Pb.d_recv + 6 * (size_t)Pb.recv_peer_off[qb], Pa.send_buf(Pa.send_cur) + 6 * (size_t)Pa.send_peer_off[qa],
                               6 * nr * sizeof(double), hipMemcpyDeviceToDevice, hb->stream) != hipSuccess)
                return PAMG_ERR_HIP;
        }
        if (pamg::launch_halo_unpack(hb->stream, hb->lv[level], hb->tov, hb->tovo) != hipSuccess) return PAMG_ERR_HIP;
        if (hipStreamSynchronize(hb->stream) != hipSuccess) return PAMG_ERR_HIP;
    }
    return PAMG_OK;
}

}  // extern "C"
