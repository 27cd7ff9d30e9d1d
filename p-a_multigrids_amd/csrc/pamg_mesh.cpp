// Mesh ingest for libpamg: gmsh 2.2 ASCII reader and neighbour search.
//
// Replaces ReadMSH (Msh2Tri.F90:132-334), whose all-pairs CheckNeig loop
// (Msh2Tri.F90:323-330, 776-963) is O(U^2) and dominates large runs
// (grofiling.txt:6-8: 99% of 792.7 s). Here candidate pairs come from an
// edge hash (O(U)), and each candidate pair (i < j) is resolved with the same
// vertex-code / direction rules as CheckNeig, in the same (i, j) order and
// with the same `no_neig == 3` early exit, so Neig / Dir / fNeig are
// identical to the reference's (tests/test_mesh.py pins them against the
// reference-generated goldens).
#include <algorithm>
#include <array>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <unordered_map>
#include <vector>

#include "pamg_internal.h"

struct pamg_mesh {
    int U = 0;
    std::vector<double> X;        // (2,3,U)
    std::vector<int> region, neig, fneig, dir;   // U, (3,U) x3
};

namespace {

struct PairHash {
    size_t operator()(const std::pair<uint64_t, uint64_t> &p) const {
        uint64_t h = p.first * 0x9E3779B97F4A7C15ull ^ (p.second + 0x632BE59BD9B4E019ull + (p.first << 6));
        return (size_t)(h ^ (h >> 29));
    }
};

uint64_t dbits(double v) {
    v = v + 0.0;   // -0.0 -> +0.0 (AreEqual treats them as equal)
    uint64_t b;
    std::memcpy(&b, &v, 8);
    return b;
}

bool trim_eq(const std::string &line, const char *tok) {
    size_t a = line.find_first_not_of(" \t\r\n");
    if (a == std::string::npos) return false;
    size_t b = line.find_last_not_of(" \t\r\n");
    return line.compare(a, b - a + 1, tok) == 0;
}

// Resolve one candidate pair exactly as CheckNeig (Msh2Tri.F90:776-963).
// vid: canonical vertex ids (coordinate-equal vertices share an id, AreEqual2).
void check_neig(pamg_mesh &m, const std::vector<int> &vid, int i, int j, int &no_neig, double l_d) {
    const double *Xi = &m.X[6 * (i - 1)], *Xj = &m.X[6 * (j - 1)];
    int counter = 0;
    for (int a = 0; a < 3 && counter <= 2; ++a)
        for (int b = 0; b < 3; ++b) {
            double dx = Xj[2 * b] - Xi[2 * a], dy = Xj[2 * b + 1] - Xi[2 * a + 1];
            if (std::sqrt(dx * dx + dy * dy) > l_d) counter += 1;
            if (counter > 2) break;
        }
    if (counter >= 2) return;
    static const int code[3][3] = {{1, 2, 3}, {2, 5, 6}, {3, 6, 9}};
    int vertex[4] = {0, 0, 0, 0};
    bool one = false, two = false, three = false, one2 = false, two2 = false, three2 = false;
    for (int a = 0; a < 3; ++a)
        for (int b = 0; b < 3; ++b)
            if (vid[3 * (i - 1) + a] == vid[3 * (j - 1) + b]) {
                vertex[a] = code[a][b];
                (a == 0 ? one : a == 1 ? two : three) = true;
                (b == 0 ? one2 : b == 1 ? two2 : three2) = true;
                break;
            }
    auto cv = [&](int num) { for (int q = 0; q < 4; ++q) if (vertex[q] == num) return true; return false; };
    int *ni = &m.neig[3 * (i - 1)], *nj = &m.neig[3 * (j - 1)];
    int *di = &m.dir[3 * (i - 1)], *dj = &m.dir[3 * (j - 1)];
    if (one && three) {
        ni[0] = j; no_neig += 1;
        if (cv(1) || (cv(2) && cv(9))) di[0] = 1;
        three = false;
    } else if (one && two) {
        ni[1] = j; no_neig += 1;
        if (cv(1) || (cv(6) && cv(2))) di[1] = 1;
        one = false;
    } else if (three && two) {
        ni[2] = j; no_neig += 1;
        if (cv(9) || (cv(6) && cv(2))) di[2] = 1;
        two = false;
    }
    int jf = (one2 && three2) ? 0 : (one2 && two2) ? 1 : (three2 && two2) ? 2 : -1;
    if (jf >= 0) {
        nj[jf] = i;
        if (one) dj[jf] = di[0];
        else if (two) dj[jf] = di[1];
        else if (three) dj[jf] = di[2];
    }
}

void build_topology(pamg_mesh &m, double l_d) {
    const int U = m.U;
    m.neig.assign(3 * (size_t)U, 0);
    m.fneig.assign(3 * (size_t)U, 0);
    m.dir.assign(3 * (size_t)U, 0);
    // canonical vertex ids by exact coordinates
    std::unordered_map<std::pair<uint64_t, uint64_t>, int, PairHash> vmap;
    vmap.reserve(3 * (size_t)U);
    std::vector<int> vid(3 * (size_t)U);
    for (int e = 0; e < U; ++e)
        for (int a = 0; a < 3; ++a) {
            auto key = std::make_pair(dbits(m.X[6 * e + 2 * a]), dbits(m.X[6 * e + 2 * a + 1]));
            auto it = vmap.emplace(key, (int)vmap.size()).first;
            vid[3 * e + a] = it->second;
        }
    // edges -> triangles (faces 1=(n1,n3), 2=(n1,n2), 3=(n2,n3))
    static const int fa[3][2] = {{0, 2}, {0, 1}, {1, 2}};
    std::unordered_map<uint64_t, std::vector<int>> edges;
    edges.reserve(3 * (size_t)U);
    for (int e = 0; e < U; ++e)
        for (int f = 0; f < 3; ++f) {
            uint64_t a = (uint64_t)vid[3 * e + fa[f][0]], b = (uint64_t)vid[3 * e + fa[f][1]];
            if (a > b) std::swap(a, b);
            edges[(a << 32) | b].push_back(e + 1);
        }
    std::vector<std::pair<int, int>> pairs;
    pairs.reserve(3 * (size_t)U);
    for (auto &kv : edges) {
        auto &v = kv.second;
        for (size_t x = 0; x < v.size(); ++x)
            for (size_t y = x + 1; y < v.size(); ++y)
                if (v[x] != v[y]) pairs.emplace_back(std::min(v[x], v[y]), std::max(v[x], v[y]));
    }
    std::sort(pairs.begin(), pairs.end());
    pairs.erase(std::unique(pairs.begin(), pairs.end()), pairs.end());
    // same visiting order as the reference's i<j double loop with its early exit
    size_t p = 0;
    while (p < pairs.size()) {
        int i = pairs[p].first, no_neig = 0;
        for (; p < pairs.size() && pairs[p].first == i; ++p) {
            if (no_neig == 3) continue;
            check_neig(m, vid, i, pairs[p].second, no_neig, l_d);
        }
    }
    // getNeigDataMesh (Msh2Tri.F90:463-468): fNeig = NumLoc(Neig(Npos), Mpos)
    for (int e = 0; e < U; ++e)
        for (int f = 0; f < 3; ++f) {
            int np = m.neig[3 * e + f], ns = 0;
            if (np != 0)
                for (int q = 0; q < 3; ++q)
                    if (m.neig[3 * (np - 1) + q] == e + 1) { ns = q + 1; break; }
            m.fneig[3 * e + f] = ns;
        }
}

double edge_len(double x1, double y1, double x2, double y2) {
    return std::sqrt((x2 - x1) * (x2 - x1) + (y2 - y1) * (y2 - y1));
}

}  // namespace

extern "C" {

int pamg_msh_read(const char *path, pamg_mesh **out) {
    if (!path || !out) return PAMG_ERR_ARG;
    std::ifstream f(path);
    if (!f) return PAMG_ERR_IO;
    std::string line;
    if (!std::getline(f, line) || !trim_eq(line, "$MeshFormat")) return PAMG_ERR_IO;
    if (!std::getline(f, line)) return PAMG_ERR_IO;
    {
        std::istringstream ss(line);
        double ver = 0; int ftype = -1;
        ss >> ver >> ftype;
        if (ftype != 0) return PAMG_ERR_IO;   // binary .msh (Msh2Tri.F90:182-186)
    }
    while (std::getline(f, line) && !trim_eq(line, "$Nodes")) {}
    if (!std::getline(f, line)) return PAMG_ERR_IO;
    long nodes = std::strtol(line.c_str(), nullptr, 10);
    if (nodes <= 0) return PAMG_ERR_IO;
    std::vector<double> vx(nodes + 1, 0.0), vy(nodes + 1, 0.0);
    for (long n = 0; n < nodes; ++n) {
        if (!std::getline(f, line)) return PAMG_ERR_IO;
        char *e1;
        long id = std::strtol(line.c_str(), &e1, 10);
        char *e2;
        double x = std::strtod(e1, &e2);
        double y = std::strtod(e2, nullptr);
        if (id < 1 || id > nodes) return PAMG_ERR_IO;
        vx[id] = x; vy[id] = y;
    }
    while (std::getline(f, line) && !trim_eq(line, "$Elements")) {}
    if (!std::getline(f, line)) return PAMG_ERR_IO;
    long nel = std::strtol(line.c_str(), nullptr, 10);
    if (nel <= 0) return PAMG_ERR_IO;
    std::vector<int> reg(nel + 1, 0);
    std::vector<std::array<long, 3>> xp(nel + 1, std::array<long, 3>{0, 0, 0});
    long skipped = 0;
    double l_d = 0.0;
    std::vector<long> tok;
    for (long e = 0; e < nel; ++e) {
        if (!std::getline(f, line)) return PAMG_ERR_IO;
        tok.clear();
        const char *c = line.c_str();
        char *end;
        for (;;) { long v = std::strtol(c, &end, 10); if (end == c) break; tok.push_back(v); c = end; }
        if (tok.size() < 3) return PAMG_ERR_IO;
        long pos = tok[0], type = tok[1];
        // triangle families kept by ReadMSH (Msh2Tri.F90:264-265)
        if (!(type == 23 || type == 21 || type == 20 || type == 9 || type == 2 || type == 24 || type == 25)) {
            skipped += 1;
            continue;
        }
        long ntag = tok[2];
        if ((long)tok.size() < 6 + ntag || pos < 1 || pos > nel) return PAMG_ERR_IO;
        reg[pos] = (int)tok[3];
        for (int k = 0; k < 3; ++k) {
            xp[pos][k] = tok[3 + ntag + k];
            if (xp[pos][k] < 1 || xp[pos][k] > nodes) return PAMG_ERR_IO;
        }
        long a = xp[pos][0], b = xp[pos][1], cc = xp[pos][2];
        l_d = std::max(l_d, edge_len(vx[a], vy[a], vx[cc], vy[cc]));
        l_d = std::max(l_d, edge_len(vx[a], vy[a], vx[b], vy[b]));
        l_d = std::max(l_d, edge_len(vx[b], vy[b], vx[cc], vy[cc]));
    }
    auto *m = new pamg_mesh;
    m->U = (int)(nel - skipped);
    m->X.assign(6 * (size_t)m->U, 0.0);
    m->region.assign(m->U, 0);
    for (long i = skipped + 1; i <= nel; ++i) {   // meshList(i-j) = meshList2(i) (:312-313)
        int e = (int)(i - skipped - 1);
        m->region[e] = reg[i];
        for (int k = 0; k < 3; ++k) {
            m->X[6 * e + 2 * k] = vx[xp[i][k]];
            m->X[6 * e + 2 * k + 1] = vy[xp[i][k]];
        }
    }
    build_topology(*m, l_d);
    *out = m;
    return PAMG_OK;
}

int pamg_msh_strip(int nx, int ny, double lx, double ly, pamg_mesh **out) {
    if (nx < 1 || ny < 1 || !out) return PAMG_ERR_ARG;
    auto *m = new pamg_mesh;
    m->U = 2 * nx * ny;
    m->X.assign(6 * (size_t)m->U, 0.0);
    m->region.assign(m->U, 11);
    double l_d = 0.0;
    int e = 0;
    for (int j = 0; j < ny; ++j)
        for (int i = 0; i < nx; ++i) {
            double x0 = lx * i / nx, x1 = lx * (i + 1) / nx, y0 = ly * j / ny, y1 = ly * (j + 1) / ny;
            const double t[2][6] = {{x0, y0, x1, y0, x0, y1}, {x1, y1, x0, y1, x1, y0}};
            for (int q = 0; q < 2; ++q, ++e)
                for (int k = 0; k < 6; ++k) m->X[6 * e + k] = t[q][k];
            l_d = std::max(l_d, edge_len(x1, y0, x0, y1));
        }
    build_topology(*m, l_d);
    *out = m;
    return PAMG_OK;
}

// gmsh 2.2 ASCII of a mesh: one node per distinct vertex (exact coordinates, %.17g: the file
// reads back bit for bit), one 3-node triangle (type 2, tags region region) per un_ele with
// its vertices in the mesh's order -- the input ReadMSH (Msh2Tri.F90:132-334) takes, so
// synthetic meshes can be fed to the reference as well
int pamg_msh_write(const pamg_mesh *m, const char *path) {
    if (!m || !path) return PAMG_ERR_ARG;
    std::unordered_map<std::pair<uint64_t, uint64_t>, int, PairHash> vmap;
    vmap.reserve(3 * (size_t)m->U);
    std::vector<int> vid(3 * (size_t)m->U);
    std::vector<int> first;   // first (element, vertex) of every node
    for (int e = 0; e < m->U; ++e)
        for (int a = 0; a < 3; ++a) {
            auto key = std::make_pair(dbits(m->X[6 * e + 2 * a]), dbits(m->X[6 * e + 2 * a + 1]));
            auto it = vmap.emplace(key, (int)vmap.size());
            if (it.second) first.push_back(3 * e + a);
            vid[3 * e + a] = it.first->second;
        }
    FILE *f = std::fopen(path, "w");
    if (!f) return PAMG_ERR_IO;
    std::fprintf(f, "$MeshFormat\n2.2 0 8\n$EndMeshFormat\n$Nodes\n%zu\n", first.size());
    for (size_t n = 0; n < first.size(); ++n)
        std::fprintf(f, "%zu %.17g %.17g 0\n", n + 1, m->X[2 * first[n]], m->X[2 * first[n] + 1]);
    std::fprintf(f, "$EndNodes\n$Elements\n%d\n", m->U);
    for (int e = 0; e < m->U; ++e)
        std::fprintf(f, "%d 2 2 %d %d %d %d %d\n", e + 1, m->region[e], m->region[e], vid[3 * e] + 1, vid[3 * e + 1] + 1,
                     vid[3 * e + 2] + 1);
    std::fprintf(f, "$EndElements\n");
    return std::fclose(f) == 0 ? PAMG_OK : PAMG_ERR_IO;
}

namespace {
// binary mesh cache: magic, version, U, FNV-1a 64 of the source file, payload, FNV-1a 64 of it
constexpr char kCacheMagic[8] = {'P', 'A', 'M', 'G', 'M', 'S', 'H', '1'};

uint64_t fnv1a(const void *p, size_t n, uint64_t h = 1469598103934665603ull) {
    const unsigned char *c = static_cast<const unsigned char *>(p);
    for (size_t i = 0; i < n; ++i) { h ^= c[i]; h *= 1099511628211ull; }
    return h;
}

int file_hash(const char *path, uint64_t *h) {
    FILE *f = std::fopen(path, "rb");
    if (!f) return PAMG_ERR_IO;
    std::vector<char> buf(1 << 20);
    uint64_t v = 1469598103934665603ull;
    size_t n;
    while ((n = std::fread(buf.data(), 1, buf.size(), f)) > 0) v = fnv1a(buf.data(), n, v);
    std::fclose(f);
    *h = v;
    return PAMG_OK;
}

uint64_t payload_hash(const pamg_mesh &m) {
    uint64_t h = fnv1a(m.X.data(), m.X.size() * sizeof(double));
    for (const auto *v : {&m.region, &m.neig, &m.fneig, &m.dir}) h = fnv1a(v->data(), v->size() * sizeof(int), h);
    return h;
}

int cache_save(const pamg_mesh &m, const char *path, uint64_t src) {
    const std::string tmp = std::string(path) + ".tmp";
    FILE *f = std::fopen(tmp.c_str(), "wb");
    if (!f) return PAMG_ERR_IO;
    const int32_t ver = 1, U = m.U;
    const uint64_t ph = payload_hash(m);
    bool ok = std::fwrite(kCacheMagic, 8, 1, f) == 1 && std::fwrite(&ver, 4, 1, f) == 1 && std::fwrite(&U, 4, 1, f) == 1 &&
              std::fwrite(&src, 8, 1, f) == 1 && std::fwrite(m.X.data(), sizeof(double), m.X.size(), f) == m.X.size();
    for (const auto *v : {&m.region, &m.neig, &m.fneig, &m.dir})
        ok = ok && std::fwrite(v->data(), sizeof(int), v->size(), f) == v->size();
    ok = ok && std::fwrite(&ph, 8, 1, f) == 1;
    ok = (std::fclose(f) == 0) && ok;
    if (!ok || std::rename(tmp.c_str(), path) != 0) { std::remove(tmp.c_str()); return PAMG_ERR_IO; }
    return PAMG_OK;
}

// loads a cache whose source hash equals `src` (src == 0: any); PAMG_ERR_STATE when stale or damaged
int cache_load(const char *path, uint64_t src, pamg_mesh **out) {
    FILE *f = std::fopen(path, "rb");
    if (!f) return PAMG_ERR_IO;
    char magic[8];
    int32_t ver = 0, U = 0;
    uint64_t s = 0, ph = 0;
    if (std::fread(magic, 8, 1, f) != 1 || std::memcmp(magic, kCacheMagic, 8) || std::fread(&ver, 4, 1, f) != 1 ||
        ver != 1 || std::fread(&U, 4, 1, f) != 1 || U < 1 || std::fread(&s, 8, 1, f) != 1 || (src && s != src)) {
        std::fclose(f);
        return PAMG_ERR_STATE;
    }
    auto *m = new pamg_mesh;
    m->U = U;
    m->X.resize(6 * (size_t)U);
    m->region.resize(U);
    m->neig.resize(3 * (size_t)U);
    m->fneig.resize(3 * (size_t)U);
    m->dir.resize(3 * (size_t)U);
    bool ok = std::fread(m->X.data(), sizeof(double), m->X.size(), f) == m->X.size();
    for (auto *v : {&m->region, &m->neig, &m->fneig, &m->dir}) ok = ok && std::fread(v->data(), sizeof(int), v->size(), f) == v->size();
    ok = ok && std::fread(&ph, 8, 1, f) == 1 && ph == payload_hash(*m);
    std::fclose(f);
    if (!ok) { delete m; return PAMG_ERR_STATE; }
    *out = m;
    return PAMG_OK;
}
}  // namespace

int pamg_msh_save(const pamg_mesh *m, const char *path) {
    if (!m || !path) return PAMG_ERR_ARG;
    return cache_save(*m, path, 0);
}

int pamg_msh_load(const char *path, pamg_mesh **m) {
    if (!path || !m) return PAMG_ERR_ARG;
    return cache_load(path, 0, m);
}

int pamg_msh_read_cached(const char *msh_path, const char *cache_path, pamg_mesh **m, int *hit) {
    if (!msh_path || !cache_path || !m) return PAMG_ERR_ARG;
    if (hit) *hit = 0;
    uint64_t h = 0;
    int rc = file_hash(msh_path, &h);
    if (rc != PAMG_OK) return rc;
    if (h == 0) h = 1;   // 0 means "any source" in the cache header
    if (cache_load(cache_path, h, m) == PAMG_OK) {
        if (hit) *hit = 1;
        return PAMG_OK;
    }
    rc = pamg_msh_read(msh_path, m);
    if (rc != PAMG_OK) return rc;
    (void)cache_save(**m, cache_path, h);   // a cache that cannot be written is not an error
    return PAMG_OK;
}

int pamg_msh_size(const pamg_mesh *m, int *U) {
    if (!m || !U) return PAMG_ERR_ARG;
    *U = m->U;
    return PAMG_OK;
}

int pamg_msh_get(const pamg_mesh *m, double *X, int *region, int *neig, int *fneig, int *dir) {
    if (!m) return PAMG_ERR_ARG;
    if (X) std::memcpy(X, m->X.data(), sizeof(double) * m->X.size());
    if (region) std::memcpy(region, m->region.data(), sizeof(int) * m->region.size());
    if (neig) std::memcpy(neig, m->neig.data(), sizeof(int) * m->neig.size());
    if (fneig) std::memcpy(fneig, m->fneig.data(), sizeof(int) * m->fneig.size());
    if (dir) std::memcpy(dir, m->dir.data(), sizeof(int) * m->dir.size());
    return PAMG_OK;
}

void pamg_msh_free(pamg_mesh *m) { delete m; }

}  // extern "C"
