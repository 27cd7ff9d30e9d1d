// VTU output of the level-1 solution: the reference's get_vtu (get_vtk_files.F90:10-165,
// called at the start of a time step, transport_tri_semi.F90:301-311) with the same
// content -- one VTK triangle (cell type 5) per level-1 sub-element with its own three
// DG nodes (points 3e..3e+2, get_splitting coordinates, Msh2Tri.F90:69-107), point data
// "Tracer" (tracer(1)%tnew), "error" (|tnew - analytical|, get_error :531-538) and
// "analytical" (boundary(x, y) = sin(x + y), splitting.F90:1401-1405) -- written at
// full fp64 precision instead of the reference's F12.10 / F10.7 / F10.3 text, either as
// raw appended binary (the default: 3 x 8 B per point and 24 B of coordinates, no
// formatting cost) or as ascii %.17g. Host code: the state comes through pamg_get_state.
#include <cmath>
#include <cinttypes>
#include <cstdio>
#include <string>
#include <vector>

#include "pamg_internal.h"

namespace {

struct Array {
    std::string name, type;
    int ncomp;
    const void *data;
    size_t count, elem;   // values, bytes per value
};

void write_ascii_values(FILE *f, const Array &a) {
    for (size_t i = 0; i < a.count; ++i) {
        if (a.type == "Float64") fprintf(f, "%.17g", static_cast<const double *>(a.data)[i]);
        else if (a.type == "Int64") fprintf(f, "%" PRId64, static_cast<const int64_t *>(a.data)[i]);
        else fprintf(f, "%u", (unsigned)static_cast<const uint8_t *>(a.data)[i]);
        fputc((i + 1) % 12 == 0 || i + 1 == a.count ? '\n' : ' ', f);
    }
}

}  // namespace

extern "C" int pamg_write_vtu(pamg_handle *h, const char *path, int ascii) {
    if (!h || !path || (ascii != 0 && ascii != 1)) return PAMG_ERR_ARG;
    if (!h->mesh_ready) return PAMG_ERR_STATE;
    const int S = h->p.n_split, U = h->U;
    const int64_t nsub = (int64_t)1 << (2 * S), ncell = nsub * U, npt = 3 * ncell;
    std::vector<double> t((size_t)npt), pts(3 * (size_t)npt), ana((size_t)npt), err((size_t)npt);
    const int rc = pamg_get_state(h, 1, PAMG_TNEW, t.data());
    if (rc != PAMG_OK) return rc;
    for (int q = 0; q < U; ++q)
        for (int e = 1; e <= nsub; ++e) {
            double xl[3][2];
            pamg::get_splitting(&h->Xo[6 * (size_t)q], S, e, xl);
            for (int i = 0; i < 3; ++i) {
                const size_t p = ((size_t)q * nsub + e - 1) * 3 + i;   // tnew(i, e, q), column-major
                pts[3 * p] = xl[i][0];
                pts[3 * p + 1] = xl[i][1];
                pts[3 * p + 2] = 0.0;
                ana[p] = std::sin(xl[i][0] + xl[i][1]);
                err[p] = std::fabs(t[p] - ana[p]);
            }
        }
    std::vector<int64_t> conn((size_t)npt), offs((size_t)ncell);
    for (int64_t p = 0; p < npt; ++p) conn[p] = p;   // ele*3-3, ele*3-2, ele*3-1 (get_vtk_files.F90:111)
    for (int64_t c = 0; c < ncell; ++c) offs[c] = 3 * (c + 1);
    std::vector<uint8_t> types((size_t)ncell, 5);      // VTK_TRIANGLE (cell_type, :119-123)
    const Array point_data[] = {{"Tracer", "Float64", 1, t.data(), (size_t)npt, 8},
                                {"error", "Float64", 1, err.data(), (size_t)npt, 8},
                                {"analytical", "Float64", 1, ana.data(), (size_t)npt, 8}};
    const Array points = {"", "Float64", 3, pts.data(), 3 * (size_t)npt, 8};
    const Array cells[] = {{"connectivity", "Int64", 1, conn.data(), (size_t)npt, 8},
                           {"offsets", "Int64", 1, offs.data(), (size_t)ncell, 8},
                           {"types", "UInt8", 1, types.data(), (size_t)ncell, 1}};
    FILE *f = fopen(path, "wb");
    if (!f) { h->err = std::string("cannot open ") + path; return PAMG_ERR_IO; }
    uint64_t offset = 0;
    auto tag = [&](const Array &a) {
        fprintf(f, "        <DataArray type=\"%s\"", a.type.c_str());
        if (!a.name.empty()) fprintf(f, " Name=\"%s\"", a.name.c_str());
        if (a.ncomp > 1) fprintf(f, " NumberOfComponents=\"%d\"", a.ncomp);
        if (ascii) {
            fprintf(f, " format=\"ascii\">\n");
            write_ascii_values(f, a);
            fprintf(f, "        </DataArray>\n");
        } else {
            fprintf(f, " format=\"appended\" offset=\"%" PRIu64 "\"/>\n", offset);
            offset += 8 + a.count * a.elem;
        }
    };
    fprintf(f, "<?xml version=\"1.0\"?>\n<VTKFile type=\"UnstructuredGrid\" version=\"1.0\" "
               "byte_order=\"LittleEndian\" header_type=\"UInt64\">\n  <UnstructuredGrid>\n"
               "    <Piece NumberOfPoints=\"%" PRId64 "\" NumberOfCells=\"%" PRId64 "\">\n"
               "      <PointData Scalars=\"Tracer\">\n", npt, ncell);
    for (const Array &a : point_data) tag(a);
    fprintf(f, "      </PointData>\n      <Points>\n");
    tag(points);
    fprintf(f, "      </Points>\n      <Cells>\n");
    for (const Array &a : cells) tag(a);
    fprintf(f, "      </Cells>\n    </Piece>\n  </UnstructuredGrid>\n");
    if (!ascii) {
        fprintf(f, "  <AppendedData encoding=\"raw\">\n   _");
        auto blob = [&](const Array &a) {
            const uint64_t n = a.count * a.elem;
            fwrite(&n, sizeof n, 1, f);
            fwrite(a.data, 1, n, f);
        };
        for (const Array &a : point_data) blob(a);
        blob(points);
        for (const Array &a : cells) blob(a);
        fprintf(f, "\n  </AppendedData>\n");
    }
    fprintf(f, "</VTKFile>\n");
    const bool ok = !ferror(f);
    if (fclose(f) != 0 || !ok) { h->err = std::string("write failed: ") + path; return PAMG_ERR_IO; }
    return PAMG_OK;
}
