// One-time setup of libpamg (host, fp64): sub-element numbering tables, the
// per-(un_ele, level) 3x3 operator records and the halo plan.
//
// Compiled with -ffp-contract=off so every quantity is formed with the
// reference's operation order (see oracle/pamg_oracle.c for the literal
// restatement these mirror); the device kernels then reproduce the
// reference's arithmetic bit for bit except the sine of the source term.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "pamg_internal.h"

namespace pamg {

// Msh2Tri.F90:32-60 get_str_info
void get_str_info(int n_split, int ele, int *irow, int *ipos, int *orientation) {
    int i = ele, row = 1, ele_row = (1 << (n_split + 1)) - 1;
    *ipos = 1; *irow = 1;
    while (i >= 1) {
        if (i > ele_row) { i -= ele_row; row += 1; ele_row -= 2; }
        else { *ipos = i; *irow = row; break; }
    }
    *orientation = *ipos % 2;
}

// splitting.F90:97-140 element_conversion (1-based fine ids)
void element_conversion(int fin[4], int coarse_ele, int i_split) {
    int irow, ipos, orient, counter, tot = 0;
    int rowx = (1 << (i_split + 1)) * 2 - 1;
    get_str_info(i_split, coarse_ele, &irow, &ipos, &orient);
    if (orient == 1) {
        counter = 2;
        while (counter < irow * 2) { tot += rowx; rowx -= 2; counter += 1; }
        fin[0] = ipos * 2 - 1 + tot;
        fin[1] = fin[0] + 1;
        fin[2] = fin[0] + 2;
        tot += rowx;
        fin[3] = ipos * 2 - 1 + tot;
    } else {
        counter = 1;
        while (counter < irow * 2) { tot += rowx; rowx -= 2; counter += 1; }
        fin[2] = (ipos / 2 - 1) * 3 + ipos / 2 + tot + 1;
        fin[1] = fin[2] + 1;
        fin[0] = fin[2] + 2;
        fin[3] = fin[0] - rowx - 2;
    }
}

// splitting.F90:427-451 loc_surf_ele_multigrid; surf(2**n, 3) column-major, 1-based values
void loc_surf_ele(int n, std::vector<int> &surf) {
    int m = 1 << n, ele, counter;
    surf.assign(3 * (size_t)m, 0);
    surf[0] = 1;
    for (ele = 2; ele <= m; ++ele) surf[ele - 1] = surf[ele - 2] + 2;
    surf[2 * m] = 1;
    counter = surf[ele - 2];
    surf[m] = counter;
    for (ele = 2; ele <= m; ++ele) {
        surf[(ele - 1) + m] = surf[(ele - 2) + m] + counter - 2;
        surf[(ele - 1) + 2 * m] = surf[(ele - 2) + m] + 1;
        counter -= 2;
    }
}

// Msh2Tri.F90:69-107 get_splitting; un_x (2,3) column-major
void get_splitting(const double *un_x, int n_split, int str_ele, double str_x[3][2]) {
    double p = (double)(1 << n_split), v1[2], v2[2];
    int irow, ipos, orient;
    v1[0] = (un_x[0] - un_x[4]) / p;
    v1[1] = (un_x[1] - un_x[5]) / p;
    v2[0] = (un_x[2] - un_x[4]) / p;
    v2[1] = (un_x[3] - un_x[5]) / p;
    get_str_info(n_split, str_ele, &irow, &ipos, &orient);
    for (int d = 0; d < 2; ++d) {
        double x3 = un_x[4 + d];
        if (ipos % 2 != 0) {
            str_x[2][d] = x3 + (irow - 1) * v2[d] + (ipos / 2) * v1[d];
            str_x[1][d] = x3 + irow * v2[d] + (ipos / 2) * v1[d];
            str_x[0][d] = x3 + (irow - 1) * v2[d] + v1[d] * (ipos / 2 + 1);
        } else {
            str_x[0][d] = x3 + irow * v2[d] + v1[d] * (ipos / 2 - 1);
            str_x[1][d] = x3 + (irow - 1) * v2[d] + v1[d] * (ipos / 2);
            str_x[2][d] = x3 + irow * v2[d] + v1[d] * (ipos / 2);
        }
    }
}

// Hierarchical storage positions (Level::pos): the coarsest level (i_split = n_split - L + 1)
// in the reference's order; on every finer level the children fin[0..3] of the coarse
// sub-element c (element_conversion) at 4 pos(c) + 0..3. pos[l] for l = 1..L, 0-based values.
void hier_positions(int n_split, int L, std::vector<int> pos[]) {
    const int ic = n_split - L + 1;
    pos[L].resize((size_t)1 << (2 * ic));
    for (size_t e = 0; e < pos[L].size(); ++e) pos[L][e] = (int)e;
    for (int l = L - 1; l >= 1; --l) {
        const int is = n_split - l + 1;
        pos[l].assign((size_t)1 << (2 * is), -1);
        for (int c = 1; c <= (1 << (2 * (is - 1))); ++c) {
            int fin[4];
            element_conversion(fin, c, is - 1);
            for (int q = 0; q < 4; ++q) pos[l][fin[q] - 1] = 4 * pos[l + 1][c - 1] + q;
        }
    }
}

// Operator record of one (un_ele, level): tri_det_nlx (ShapFun.F90:1389-1454) scaled by
// semi_tri_det_nlx_multigrid (:1678-1683), get_un_ele_mass_stiff_diffvol
// (ShapFun_unstruc.F90:304-335), the diff_vol1 reduction (transport_tri_semi.F90:602-606)
// and get_diagonal (:481-486). The quadrature is TRIQUAold's ngi=3 edge-midpoint rule
// (ShapFun.F90:554-563) with SHATRIold's P1 functions (:1036-1048).
void level_stencil(const double *X, int i_split, double k, double dt, double omega, double *rec, double *D0) {
    static const double N[3][3] = {{0.5, 0.5, 0.0}, {0.0, 0.5, 0.5}, {0.5, 0.0, 0.5}};
    static const double NLX[2][3] = {{1.0, 0.0, -1.0}, {0.0, 1.0, -1.0}};
    const double weight = 1.0 / 3.0;
    double detwei[3], nx[3][2][3];
    for (int g = 0; g < 3; ++g) {
        double agi = 0, bgi = 0, cgi = 0, dgi = 0;
        for (int L = 0; L < 3; ++L) {
            agi = agi + NLX[0][L] * X[2 * L];
            bgi = bgi + NLX[0][L] * X[2 * L + 1];
            cgi = cgi + NLX[1][L] * X[2 * L];
            dgi = dgi + NLX[1][L] * X[2 * L + 1];
        }
        double detj = agi * dgi - bgi * cgi;
        detwei[g] = 0.5 * std::fabs(detj) * weight;
        double a11 = dgi / detj, a21 = -(cgi / detj), a12 = -(bgi / detj), a22 = agi / detj;
        for (int L = 0; L < 3; ++L) {
            nx[g][0][L] = a11 * NLX[0][L] + a12 * NLX[1][L];
            nx[g][1][L] = a21 * NLX[0][L] + a22 * NLX[1][L];
        }
        detwei[g] = detwei[g] / (double)(1 << (2 * i_split));
        for (int d = 0; d < 2; ++d)
            for (int L = 0; L < 3; ++L) nx[g][d][L] = nx[g][d][L] * (double)(1 << i_split);
    }
    double ml[3], M[3][3], Kd[3][3];
    for (int j = 0; j < 3; ++j) {
        double s = 0;
        for (int g = 0; g < 3; ++g) s = s + N[g][j] * detwei[g];
        ml[j] = s;
        for (int i = 0; i < 3; ++i) {
            double m = 0;
            for (int g = 0; g < 3; ++g) m = m + N[g][i] * detwei[g] * N[g][j];
            M[i][j] = m;
        }
    }
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            double acc = 0.0;
            for (int d = 0; d < 2; ++d) {
                double s = 0;
                for (int g = 0; g < 3; ++g) s = s + k * nx[g][d][i] * detwei[g] * nx[g][d][j];
                acc = acc + s;
            }
            Kd[i][j] = acc;
        }
    std::memset(rec, 0, sizeof(double) * kStcStride);
    double rdt = 1 / dt;
    for (int i = 0; i < 3; ++i) {
        for (int j = 0; j < 3; ++j) {
            rec[kStcM + 3 * i + j] = M[i][j];
            rec[kStcK + 3 * i + j] = Kd[i][j];
        }
        double D = rdt * ml[i] + Kd[i][i] + 0.0;
        rec[kStcW + i] = omega / D;
        if (D0) D0[i] = D;
        for (int j = 0; j < 3; ++j) rec[kStcA + 3 * i + j] = rdt * M[i][j] + Kd[i][j];
    }
    rec[kStcC] = M[0][1];
    rec[kStcOm] = omega;
}

bool mass_is_p1_midpoint(const double *rec) {
    const double c = rec[kStcC];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
            if (rec[kStcM + 3 * i + j] != (i == j ? 2.0 * c : c)) return false;
    return true;
}

// Halo plan of update_overlaps (splitting.F90:1210-1397) for level l:
// for every owned un_ele u, faces in the order 1, 3, 2, and the 2**i boundary
// sub-elements surf_ele(:, f): either a boundary-condition write of
// sin(x+y) at two nodes into u's own t_overlap(:, f), or a copy of
// (tnew, told)(:, s, u) into t_overlap(slot, Nside) of the neighbour.
// Each destination word has exactly one writer, so the plan is order-free.
int build_halo(pamg_handle *h, int l, const double *Xg, const int *neig, const int *fneig, const int *dir) {
    Level &L = h->lv[l];
    HaloPlan &P = L.halo;
    P.local.clear(); P.bc.clear(); P.remote.clear(); P.recv_dst.clear();
    P.peers.clear(); P.send_peer_off.clear(); P.recv_peer_off.clear();
    P.hface.assign((size_t)h->U * 3, make_int4(0, 0, 0, 0));
    P.bcv.clear();
    const int is = L.isplit, m = 1 << is, sl = h->slots;
    std::vector<int> &surf = P.surf;
    loc_surf_ele(is, surf);
    P.n_told = 0;
    // storage position of the reference's sub-element se (Level::pos; identity when none is
    // set: the host-only plan of pamg_plan_build reports the reference's numbering)
    auto spos = [&](int se) { return L.pos.empty() ? se - 1 : L.pos[se - 1]; };
    P.hsub.assign(L.nsub, make_int4(0, 0, 0, 0));
    for (int f = 1; f <= 3; ++f)
        for (int i = 1; i <= m; ++i) {
            int4 &e = P.hsub[spos(surf[(i - 1) + (f - 1) * m])];
            (f == 1 ? e.x : f == 2 ? e.y : e.z) = i;
        }
    std::vector<std::pair<int, int>> remote_block((size_t)h->U * 3, std::make_pair(-1, -1));   // (peer, first index)
    const bool dist = !h->owner.empty();
    const bool selfp = dist && !h->vpart.empty();
    std::vector<int> g2l;   // global -> local index (or -1)
    if (dist) {
        g2l.assign(h->U_global, -1);
        for (int q = 0; q < h->U; ++q) g2l[h->owned[q]] = q;
    }
    // remote entries grouped by destination rank, in (sender u, face, i) order
    std::vector<std::vector<HaloCopy>> by_peer(h->nranks);
    static const int face_order[3] = {1, 3, 2};
    for (int q = 0; q < h->U; ++q) {
        const int ug = dist ? h->owned[q] : q;
        const double *X = Xg + 6 * (size_t)ug;
        for (int fo = 0; fo < 3; ++fo) {
            const int f = face_order[fo];
            for (int i = 1; i <= m; ++i) {
                const int se = surf[(i - 1) + (f - 1) * m];
                int irow, ipos, orient;
                get_str_info(is, se, &irow, &ipos, &orient);
                if ((f == 1 && (irow != 1 || ipos != 2 * i - 1)) || (f != 1 && irow != i)) {
                    h->err = "halo: unexpected boundary sub-element numbering";
                    return PAMG_ERR_STATE;
                }
                const int npos = neig[3 * (size_t)ug + f - 1];
                const int src = q * L.nsub + spos(se);
                if (npos == 0) {
                    double xl[3][2];
                    get_splitting(X, is, se, xl);
                    int a, b, na, nb;
                    if (f == 1) { a = (ipos / 2) * 3 + 1; b = (ipos / 2) * 3 + 3; na = 0; nb = 2; }
                    else if (f == 3) { a = (irow - 1) * 3 + 2; b = (irow - 1) * 3 + 3; na = 1; nb = 2; }
                    else { a = (irow - 1) * 3 + 1; b = (irow - 1) * 3 + 2; na = 0; nb = 1; }
                    const int base = q * sl * 3 + (f - 1) * sl;
                    HaloBC e;
                    e.dst_a = base + a - 1;
                    e.dst_b = base + b - 1;
                    e.val_a = std::sin(xl[na][0] + xl[na][1]);   // boundary(), splitting.F90:1401-1405
                    e.val_b = std::sin(xl[nb][0] + xl[nb][1]);
                    if (i == 1) P.hface[3 * (size_t)q + f - 1] = make_int4(0, base, (int)P.bc.size(), 0);
                    P.bc.push_back(e);
                    P.bcv.push_back(make_double2(e.val_a, e.val_b));
                } else {
                    const int nside = fneig[3 * (size_t)ug + f - 1];
                    const int dr = dir[3 * (size_t)ug + f - 1];
                    if (nside < 1 || nside > 3) {
                        h->err = "halo: asymmetric neighbour table (fNeig = 0) at un_ele " + std::to_string(ug + 1);
                        return PAMG_ERR_ARG;
                    }
                    int fwd, rev;
                    if (f == 1) { fwd = ipos / 2 + 1; rev = m - (ipos / 2 + 1) + 1; }
                    else { fwd = irow; rev = m - irow + 1; }
                    if (f == 2) std::swap(fwd, rev);   // face 2 branches are mirrored (:1354-1391)
                    const int kslot = (nside == 2) ? (dr ? rev : fwd) : (dr ? fwd : rev);
                    const int ng = npos - 1;
                    const int off_in_elem = (nside - 1) * sl + kslot * 3 - 3;
                    // kslot is i or m - i + 1 (surf_ele(i, f) sits at ipos = 2i-1 on face 1 and in row i on faces 2, 3)
                    const int rev_flag = (kslot == i) ? 0 : 1;
                    if (kslot != i && kslot != m - i + 1) { h->err = "halo: slot map"; return PAMG_ERR_STATE; }
                    // self-peer plan (pamg_comm_init_self): a face between two virtual parts is a
                    // remote face whose peer is this rank itself
                    const bool remote = selfp ? h->vpart[ng] != h->vpart[ug] : (dist && h->owner[ng] != h->rank);
                    const int peer = selfp ? h->rank : (dist ? h->owner[ng] : 0);
                    if (!remote) {
                        const int nl = dist ? g2l[ng] : ng;
                        if (i == 1) {
                            P.hface[3 * (size_t)q + f - 1] =
                                make_int4(1 | (rev_flag << 2), nl * sl * 3 + (nside - 1) * sl, 0, P.n_told);
                            P.n_told += m;
                        }
                        P.local.push_back(HaloCopy{src, nl * sl * 3 + off_in_elem});
                    } else {
                        if (i == 1) {
                            remote_block[3 * (size_t)q + f - 1] = std::make_pair(peer, (int)by_peer[peer].size());
                            P.hface[3 * (size_t)q + f - 1] = make_int4(2, 0, 0, P.n_told);
                            P.n_told += m;
                        }
                        by_peer[peer].push_back(HaloCopy{src, off_in_elem});
                    }
                }
            }
        }
    }
    if (dist) {
        // send side: peers in ascending rank order
        P.send_peer_off.push_back(0);
        for (int r = 0; r < h->nranks; ++r) {
            if (r == h->rank && !selfp) continue;
            bool has_send = !by_peer[r].empty();
            // receive side from r: enumerate r's owned elements in the same order
            std::vector<int> rd;
            for (int ug = 0; ug < h->U_global; ++ug) {
                if (h->owner[ug] != r) continue;
                for (int fo = 0; fo < 3; ++fo) {
                    const int f = face_order[fo];
                    const int npos = neig[3 * (size_t)ug + f - 1];
                    if (npos == 0 || h->owner[npos - 1] != h->rank) continue;
                    if (selfp && h->vpart[npos - 1] == h->vpart[ug]) continue;
                    const int nside = fneig[3 * (size_t)ug + f - 1];
                    const int dr = dir[3 * (size_t)ug + f - 1];
                    for (int i = 1; i <= m; ++i) {
                        const int se = surf[(i - 1) + (f - 1) * m];
                        int irow, ipos, orient;
                        get_str_info(is, se, &irow, &ipos, &orient);
                        int fwd, rev;
                        if (f == 1) { fwd = ipos / 2 + 1; rev = m - (ipos / 2 + 1) + 1; }
                        else { fwd = irow; rev = m - irow + 1; }
                        if (f == 2) std::swap(fwd, rev);
                        const int kslot = (nside == 2) ? (dr ? rev : fwd) : (dr ? fwd : rev);
                        const int nl = g2l[npos - 1];
                        rd.push_back(nl * sl * 3 + (nside - 1) * sl + kslot * 3 - 3);
                    }
                }
            }
            if (!has_send && rd.empty()) continue;
            P.peers.push_back(r);
            const int first = (int)P.remote.size();
            for (size_t b = 0; b < remote_block.size(); ++b)
                if (remote_block[b].first == r) P.hface[b].z = first + remote_block[b].second;
            for (auto &e : by_peer[r]) P.remote.push_back(HaloCopy{e.src, (int)P.remote.size()});
            P.send_peer_off.push_back((int)P.remote.size());
            if (P.recv_peer_off.empty()) P.recv_peer_off.push_back(0);
            P.recv_dst.insert(P.recv_dst.end(), rd.begin(), rd.end());
            P.recv_peer_off.push_back((int)P.recv_dst.size());
        }
        if (P.recv_peer_off.empty()) P.recv_peer_off.push_back(0);
    }
    // the device's surf table (k_told_halo, k_overlap_static) holds storage positions, 1-based
    for (int &v : surf) v = spos(v) + 1;
    return PAMG_OK;
}


// ---- the face-coupled operator (pamg_params.op = 1; oracle/pamg_oracle.c face_setup
// is the restatement these tables follow, operation for operation)
namespace {
const int kFNode[3][2] = {{1, 3}, {3, 2}, {2, 1}};   // face_nodes (transport_tri_semi.F90:142-147)
const int kFMface[3] = {1, 3, 2};                     // un_ele face of sub-element face f (:626-637)

// splitting.F90:732-776 get_str_neig_multigrid: sn[(f - 1) + 3 (e - 1)]
void get_str_neig(int n, std::vector<int> &sn) {
    int total = (1 << (n + 1)) - 1, current = total, irow = (1 << n) - 1, ele;
    sn.assign(3 * ((size_t)1 << (2 * n)) + 3, 0);
    auto SN = [&](int f, int e) -> int & { return sn[(f - 1) + 3 * (size_t)(e - 1)]; };
    SN(1, 1) = 0; SN(2, 1) = 0; SN(3, 1) = 2;
    ele = 2;
    while (ele <= total) {
        SN(2, ele) = ele + 1; SN(3, ele) = ele - 1; SN(1, ele) = ele + total - 1;
        ele = ele + 1;
        SN(2, ele) = ele - 1; SN(1, ele) = 0; SN(3, ele) = ele + 1;
        ele = ele + 1;
    }
    SN(3, ele - 1) = 0;
    while (irow >= 1) {
        total = total + current - 2;
        current = current - 2;
        SN(2, ele) = 0; SN(3, ele) = ele + 1; SN(1, ele) = ele - current - 1;
        ele = ele + 1;
        while (ele <= total) {
            SN(2, ele) = ele + 1; SN(3, ele) = ele - 1; SN(1, ele) = ele + current - 1;
            ele = ele + 1;
            SN(2, ele) = ele - 1; SN(3, ele) = ele + 1; SN(1, ele) = ele - current - 1;
            ele = ele + 1;
        }
        SN(3, ele - 1) = 0;
        irow = irow - 1;
    }
}

double dist2d(const double a[2], const double b[2]) {
    double dx = a[0] - b[0], dy = a[1] - b[1];
    return std::sqrt(dx * dx + dy * dy);
}
void centroid(double xl[3][2], double c[2]) {
    for (int d = 0; d < 2; ++d) c[d] = (xl[0][d] + xl[1][d] + xl[2][d]) / 3.0;
}
double face_weight(double k, double delta, double len) { return k / delta * len / 6.0; }

// the slot update_overlaps gives the sub-element at position i of face f of un_ele q (splitting.F90:1297-1391)
int overlap_kslot(int is, const std::vector<int> &surf, int f, int i, int nside, int dr) {
    const int m = 1 << is;
    int irow, ipos, orient, fwd, rev;
    get_str_info(is, surf[(i - 1) + (f - 1) * m], &irow, &ipos, &orient);
    if (f == 1) { fwd = ipos / 2 + 1; rev = m - (ipos / 2 + 1) + 1; }
    else { fwd = irow; rev = m - irow + 1; }
    if (f == 2) std::swap(fwd, rev);
    return (nside == 2) ? (dr ? rev : fwd) : (dr ? fwd : rev);
}
}  // namespace

int build_face(pamg_handle *h, int l, const double *Xg, const int *neig, const int *fneig, const int *dir,
               std::vector<int4> &fnb, std::vector<double> &fface, std::vector<int> &fsx) {
    Level &L = h->lv[l];
    const int is = L.isplit, nsub = L.nsub, m = 1 << is;
    std::vector<int> sn, surf;
    get_str_neig(is, sn);
    loc_surf_ele(is, surf);
    fnb.assign(nsub, make_int4(0, 0, 0, 0));
    for (int e = 1; e <= nsub; ++e) {
        int irow, ipos, orient, v[3];
        get_str_info(is, e, &irow, &ipos, &orient);
        for (int f = 1; f <= 3; ++f) {
            const int nb = sn[(f - 1) + 3 * (size_t)(e - 1)];
            v[f - 1] = nb ? L.pos[nb - 1] : -((f == 1) ? ipos / 2 + 1 : irow);
        }
        fnb[L.pos[e - 1]] = make_int4(v[0], v[1], v[2], ipos % 2);
    }
    fface.assign((size_t)std::max(h->U, 1) * kFaceStride, 0.0);
    fsx.assign((size_t)std::max(h->U, 1) * 4, 0);
    for (int q = 0; q < h->U; ++q) {
        const int ug = h->owned.empty() ? q : h->owned[q];
        const double *X = Xg + 6 * (size_t)ug;
        double *w = &fface[(size_t)q * kFaceStride];
        for (int f = 1; f <= 3; ++f)   // inner faces: the first up sub-element with a neighbour across f
            for (int e = 1; e <= nsub; ++e) {
                int irow, ipos, orient;
                const int nb = sn[(f - 1) + 3 * (size_t)(e - 1)];
                get_str_info(is, e, &irow, &ipos, &orient);
                if (!(ipos % 2) || !nb) continue;
                double xe[3][2], xn[3][2], ce[2], cn[2];
                get_splitting(X, is, e, xe);
                get_splitting(X, is, nb, xn);
                centroid(xe, ce);
                centroid(xn, cn);
                w[f - 1] = face_weight(h->p.k, dist2d(ce, cn), dist2d(xe[kFNode[f - 1][0] - 1], xe[kFNode[f - 1][1] - 1]));
                break;
            }
        for (int fi = 0; fi < 3; ++fi) {   // un_ele faces, from the boundary sub-element at sp = 1
            const int mface = kFMface[fi], se = surf[0 + (mface - 1) * m];
            const int a = kFNode[fi][0], b = kFNode[fi][1];
            double xe[3][2], ce[2];
            get_splitting(X, is, se, xe);
            centroid(xe, ce);
            const double len = dist2d(xe[a - 1], xe[b - 1]);
            const int npos = neig[3 * (size_t)ug + mface - 1];
            if (npos == 0) {
                const double mid[2] = {(xe[a - 1][0] + xe[b - 1][0]) / 2.0, (xe[a - 1][1] + xe[b - 1][1]) / 2.0};
                w[3 + mface - 1] = face_weight(h->p.k, dist2d(ce, mid), len);
                fsx[4 * (size_t)q + mface - 1] = a | (b << 2) | (1 << 4);
                continue;
            }
            const int nq = npos - 1, nside = fneig[3 * (size_t)ug + mface - 1];
            bool found = false;
            for (int i = 1; i <= m && !found; ++i) {
                if (overlap_kslot(is, surf, nside, i, fneig[3 * (size_t)nq + nside - 1], dir[3 * (size_t)nq + nside - 1]) != 1)
                    continue;
                double xn[3][2], cn[2];
                get_splitting(Xg + 6 * (size_t)nq, is, surf[(i - 1) + (nside - 1) * m], xn);
                centroid(xn, cn);
                int S[2] = {0, 0};
                for (int t = 0; t < 2; ++t) {
                    const double *p = xe[(t ? b : a) - 1];
                    double best = 1e300;
                    for (int r = 0; r < 3; ++r) {
                        const double d = dist2d(p, xn[r]);
                        if (d < best) { best = d; S[t] = r + 1; }
                    }
                    if (best > 1e-9 * len) {
                        h->err = "face operator: the halo slot of un_ele " + std::to_string(ug + 1) + " face " +
                                 std::to_string(mface) + " holds no sub-element sharing that face";
                        return PAMG_ERR_STATE;
                    }
                }
                w[3 + mface - 1] = face_weight(h->p.k, dist2d(ce, cn), len);
                fsx[4 * (size_t)q + mface - 1] = S[0] | (S[1] << 2);
                found = true;
            }
            if (!found) { h->err = "face operator: no halo slot 1 on a neighbour's face"; return PAMG_ERR_STATE; }
        }
        double rec[kStcStride];
        level_stencil(X, is, h->p.k, h->p.dt, h->p.omega, rec, w + 6);   // D0 = rdt ml + Kd_ii + 0.0
        // omega / D for each pattern of inner faces (get_diagonal's surface term, :481-486): D_i =
        // D0_i + 2 w_f over the faces containing node i, in face order, as the oracle's face_terms
        for (int pt = 0; pt < 8; ++pt) {
            double D[3] = {w[6], w[7], w[8]};
            for (int fi = 0; fi < 3; ++fi) {
                const int a = kFNode[fi][0] - 1, b = kFNode[fi][1] - 1;
                const double wf = ((pt >> fi) & 1) ? w[fi] : w[3 + kFMface[fi] - 1];
                D[a] = D[a] + 2.0 * wf;
                D[b] = D[b] + 2.0 * wf;
            }
            for (int i = 0; i < 3; ++i) w[kFaceWD + 3 * pt + i] = h->p.omega / D[i];
        }
    }
    return PAMG_OK;
}

}  // namespace pamg
