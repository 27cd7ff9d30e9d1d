/*
 * ORACLE TEST INFRASTRUCTURE -- not product code.
 *
 * CPU restatement (plain C, fp64, scalar, single thread) of the reference's
 * live multigrid path: the mode-9 driver `Semi_implicit_iterative`
 * (transport_tri_semi.F90:14-891, selected by main.F90:16,46-47) with its
 * internal smoother / get_residual / get_A_x / get_RHS / get_diagonal /
 * solve_* subroutines, the inter-level transfers restrictor / prolongator /
 * element_conversion (splitting.F90:10-151), the halo update_overlaps
 * (splitting.F90:1210-1397), the sub-element numbering and geometry
 * get_str_info / get_splitting (Msh2Tri.F90:32-107), the gmsh reader and the
 * neighbour search ReadMSH / CheckNeig / getNeigDataMesh
 * (Msh2Tri.F90:132-334,454-548,776-963) and the per-level shape-function
 * scaling tri_det_nlx / semi_tri_det_nlx_multigrid (ShapFun.F90:1389-1454,
 * 1661-1684) plus get_un_ele_mass_stiff_diffvol (ShapFun_unstruc.F90:304-335).
 *
 * It is the parity checker for the HIP path and the "port" CPU baseline.
 * It follows the reference's structure literally -- stencils re-derived per
 * un_ele per pass, source term and level-1 RHS re-evaluated at every
 * sub-element visit, halo rewritten at the start of every sweep, the
 * tnew / tnew_nonlin state machine of transport_tri_semi.F90:299-381 -- and
 * its floating-point operation order (compile with -ffp-contract=off).
 * Pinned against the instrumented reference build (oracle/build_ref.py) by
 * tests/test_oracle_golden.py.
 *
 * Data layout = the reference's Fortran arrays: a level field
 * tracer(l)%x(3, nsub_l, U) column-major is a C array [U][nsub_l][3].
 * Quantities the reference leaves uninitialised are defined as zero (see
 * oracle/build_ref.py for the matching patches).
 */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define NLOC 3
#define NGI 3

/* The per-un_ele loops of the mode-9 path are independent (block-diagonal operator; every halo
 * word has one writer), so the checker splits them over OpenMP threads when built with
 * -fopenmp: the results are the same bits for any thread count. */
#ifdef _OPENMP
#define PAMG_ORC_PARALLEL _Pragma("omp parallel for schedule(static)")
#else
#define PAMG_ORC_PARALLEL
#endif

typedef struct {
    int n_split, levels, n_smooth, n_coarse, solver, ntime, n_multigrid;
    double dt, k, omega, theta;
    int coarse_solver;   /* 0: the reference (:351-353); 1: exact local solve (the build's direct path) */
    int op;              /* 0: the reference's mode-9 operator (block diagonal); 1: the face-coupled
                            interior-penalty operator of SURVEY.md 8(f) rank 1 (face_* below) */
    int arith;           /* 0: the reference's operation order; 1: the build's contracted arithmetic
                            (pamg_params.arith = 1): A_e = rdt M + Kd formed once, one fma chain per
                            row -- the same algebra, other roundings; checks the HIP path's arith = 1
                            bit for bit (solvers 1 / 3) */
} orc_cfg;

typedef struct {
    orc_cfg c;
    int U;
    double *X;      /* (2,3,U) */
    int *region;    /* U */
    int *neig;      /* (3,U), 1-based, 0 = boundary */
    int *fneig;     /* (3,U) */
    int *dir;       /* (3,U) 0/1 */
    int nsub[16];   /* 4^(S-l+1), index l-1 */
    double *tnew[16], *told[16], *rhs[16], *res[16], *source[16];
    double *tnn;    /* tnew_nonlin, shape of level tnn_level */
    int tnn_level;
    double *detwei[16]; /* (3,U) per level */
    double *nx[16];     /* (ngi,2,3,U) per level */
    double *t_overlap, *t_overlap_old; /* (2^S*3, 3, U) */
    int slots;
    /* test hook (orc_set_source): level 1's cascaded source term s' taken from here instead of
     * being evaluated with the host libm sin -- so that a comparison with the HIP path, whose
     * device sin may differ in the last bit, can be bitwise everywhere else */
    double *src_override;
    /* op = 1, per level: fnb (nsub, 3) the neighbour str_ele across each face (> 0) or -sp (the
     * sub-element's position along its un_ele face, < 0); fw (U, 9) the face weights w_in[3] (inner
     * faces by face index), w_b[3] (un_ele faces 1..3) and D0[3] = rdt ml + Kd_ii; fsx (U, 3) per
     * un_ele face the neighbour-local nodes S(F1) | S(F2) << 2 holding the values at my face nodes */
    int *fnb[16];
    double *fw[16];
    int *fsx[16];
} orc_state;

/* ---------------------------------------------------------------- helpers */

/* Msh2Tri.F90:32-60 get_str_info */
static void get_str_info(int n_split, int ele, int *irow, int *ipos, int *orientation) {
    int i = ele, row = 1, ele_row = (1 << (n_split + 1)) - 1;
    while (i >= 1) {
        if (i > ele_row) { i -= ele_row; row += 1; ele_row -= 2; }
        else { *ipos = i; *irow = row; break; }
    }
    *orientation = *ipos % 2;
}

/* Msh2Tri.F90:69-107 get_splitting; un_x is (2,3) column-major */
static void get_splitting(const double *un_x, int n_split, int str_ele, double str_x[3][2]) {
    double p = (double)(1 << n_split);
    double v1[2], v2[2];
    int irow = 0, ipos = 0, orient = 0;
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

/* splitting.F90:1401-1405 boundary */
static double boundary(double a, double b) { return sin(a + b); }

/* splitting.F90:97-140 element_conversion; fin_ele 1-based */
static void element_conversion(int fin[4], int coarse_ele, int i_split) {
    int irow = 0, ipos = 0, orient = 0, counter, tot_fine = 0;
    int rowx = (1 << (i_split + 1)) * 2 - 1;
    get_str_info(i_split, coarse_ele, &irow, &ipos, &orient);
    if (orient == 1) {
        counter = 2;
        while (counter < irow * 2) { tot_fine += rowx; rowx -= 2; counter += 1; }
        fin[0] = ipos * 2 - 1 + tot_fine;
        fin[1] = fin[0] + 1;
        fin[2] = fin[0] + 2;
        tot_fine += rowx;
        fin[3] = ipos * 2 - 1 + tot_fine;
    } else {
        counter = 1;
        while (counter < irow * 2) { tot_fine += rowx; rowx -= 2; counter += 1; }
        fin[2] = (ipos / 2 - 1) * 3 + ipos / 2 + tot_fine + 1;
        fin[1] = fin[2] + 1;
        fin[0] = fin[2] + 2;
        fin[3] = fin[0] - rowx - 2;
    }
}

/* splitting.F90:427-451 loc_surf_ele_multigrid; surf is (2^n, 3) column-major, 1-based values */
static void loc_surf_ele(int n, int *surf) {
    int m = 1 << n, ele, counter;
    surf[0 + 0 * m] = 1;
    for (ele = 2; ele <= m; ++ele) surf[(ele - 1) + 0 * m] = surf[(ele - 2) + 0 * m] + 2;
    surf[0 + 2 * m] = 1;
    counter = surf[(ele - 2) + 0 * m];
    surf[0 + 1 * m] = counter;
    for (ele = 2; ele <= m; ++ele) {
        surf[(ele - 1) + 1 * m] = surf[(ele - 2) + 1 * m] + counter - 2;
        surf[(ele - 1) + 2 * m] = surf[(ele - 2) + 1 * m] + 1;
        counter -= 2;
    }
}

/* --------------------------------------------------------- mesh ingest */

typedef struct { int nodes; double *vx, *vy; } vtx_t;

static int next_line(FILE *f, char *buf, int n) { return fgets(buf, n, f) != NULL; }

static int trim_eq(const char *line, const char *tok) {
    size_t n = strlen(tok);
    while (*line == ' ' || *line == '\t') ++line;
    if (strncmp(line, tok, n)) return 0;
    line += n;
    while (*line == ' ' || *line == '\t' || *line == '\r' || *line == '\n') ++line;
    return *line == 0;
}

/* Generic.F90:50-58 AreEqual2: |X-Y|_2 < epsilon(double) */
static int are_equal(double ax, double ay, double bx, double by) {
    double dx = ax - bx, dy = ay - by;
    return sqrt(dx * dx + dy * dy) < 2.220446049250313e-16;
}

static int check_vector(const int v[4], int num) {
    for (int i = 0; i < 4; ++i) if (v[i] == num) return 1;
    return 0;
}

static double length2d(double x1, double y1, double x2, double y2) {
    return sqrt((x2 - x1) * (x2 - x1) + (y2 - y1) * (y2 - y1));
}

/* Msh2Tri.F90:776-963 CheckNeig (literal, including the l_d pre-filter) */
static void check_neig(orc_state *s, int i, int j, int *no_neig, double l_d) {
    const double *Xi = s->X + 6 * (i - 1), *Xj = s->X + 6 * (j - 1);
    int vertex[4] = {0, 0, 0, 0}, counter = 0;
    int one = 0, two = 0, three = 0, one2 = 0, two2 = 0, three2 = 0;
    for (int a = 0; a < 3; ++a) {
        for (int b = 0; b < 3; ++b) {
            double d = length2d(Xi[2 * a], Xi[2 * a + 1], Xj[2 * b], Xj[2 * b + 1]);
            if (d > l_d) counter += 1;
            if (counter > 2) break;
        }
        if (counter > 2) break;
    }
    if (counter >= 2) return;
    /* vertex codes as assigned at Msh2Tri.F90:820-871 */
    static const int code[3][3] = {{1, 2, 3}, {2, 5, 6}, {3, 6, 9}};
    for (int a = 0; a < 3; ++a) {
        for (int b = 0; b < 3; ++b) {
            if (are_equal(Xi[2 * a], Xi[2 * a + 1], Xj[2 * b], Xj[2 * b + 1])) {
                vertex[a] = code[a][b];
                if (a == 0) one = 1; else if (a == 1) two = 1; else three = 1;
                if (b == 0) one2 = 1; else if (b == 1) two2 = 1; else three2 = 1;
                break;
            }
        }
    }
    int *ni = s->neig + 3 * (i - 1), *nj = s->neig + 3 * (j - 1);
    int *di = s->dir + 3 * (i - 1), *dj = s->dir + 3 * (j - 1);
    if (one && three) {
        ni[0] = j; *no_neig += 1;
        if (check_vector(vertex, 1) || (check_vector(vertex, 2) && check_vector(vertex, 9))) di[0] = 1;
        three = 0;
    } else if (one && two) {
        ni[1] = j; *no_neig += 1;
        if (check_vector(vertex, 1) || (check_vector(vertex, 6) && check_vector(vertex, 2))) di[1] = 1;
        one = 0;
    } else if (three && two) {
        ni[2] = j; *no_neig += 1;
        if (check_vector(vertex, 9) || (check_vector(vertex, 6) && check_vector(vertex, 2))) di[2] = 1;
        two = 0;
    }
    int jf = -1;
    if (one2 && three2) jf = 0;
    else if (one2 && two2) jf = 1;
    else if (three2 && two2) jf = 2;
    if (jf >= 0) {
        nj[jf] = i;
        if (one) dj[jf] = di[0];
        else if (two) dj[jf] = di[1];
        else if (three) dj[jf] = di[2];
    }
}

/* Msh2Tri.F90:132-334 ReadMSH (gmsh 2.2 ascii). Returns number of triangles
 * or <0 on error; if s != NULL also fills s->X, region, neig, dir, fneig. */
static int read_msh(const char *path, orc_state *s) {
    FILE *f = fopen(path, "r");
    if (!f) return -1;
    char line[4096];
    int nodes = 0, nel = 0;
    double *vx = NULL, *vy = NULL;
    while (next_line(f, line, sizeof line)) if (trim_eq(line, "$Nodes")) break;
    if (!next_line(f, line, sizeof line)) { fclose(f); return -2; }
    nodes = atoi(line);
    vx = calloc(nodes + 1, sizeof(double)); vy = calloc(nodes + 1, sizeof(double));
    for (int i = 0; i < nodes; ++i) {
        int id; double x, y, z;
        if (!next_line(f, line, sizeof line) || sscanf(line, "%d %lf %lf %lf", &id, &x, &y, &z) != 4 ||
            id < 1 || id > nodes) { fclose(f); free(vx); free(vy); return -3; }
        vx[id] = x; vy[id] = y;
    }
    while (next_line(f, line, sizeof line)) if (trim_eq(line, "$Elements")) break;
    if (!next_line(f, line, sizeof line)) { fclose(f); free(vx); free(vy); return -4; }
    nel = atoi(line);
    int *pos_of = calloc(nel + 1, sizeof(int)), *reg = calloc(nel + 1, sizeof(int));
    int (*xp)[3] = calloc(nel + 1, sizeof *xp);
    int j = 0;
    double l_d = 0.0;
    for (int i = 0; i < nel; ++i) {
        if (!next_line(f, line, sizeof line)) { fclose(f); return -5; }
        int tok[64], nt = 0;
        char *p = line, *end;
        while (nt < 64) { long v = strtol(p, &end, 10); if (end == p) break; tok[nt++] = (int)v; p = end; }
        int pos = tok[0], type = tok[1];
        if (!(type == 23 || type == 21 || type == 20 || type == 9 || type == 2 || type == 24 || type == 25)) {
            j += 1; continue;
        }
        int ntag = tok[2];
        reg[pos] = tok[3];
        xp[pos][0] = tok[3 + ntag]; xp[pos][1] = tok[4 + ntag]; xp[pos][2] = tok[5 + ntag];
        int a = xp[pos][0], b = xp[pos][1], c = xp[pos][2];
        double d1 = length2d(vx[a], vy[a], vx[c], vy[c]);
        double d2 = length2d(vx[a], vy[a], vx[b], vy[b]);
        double d3 = length2d(vx[b], vy[b], vx[c], vy[c]);
        if (d1 > l_d) l_d = d1;
        if (d2 > l_d) l_d = d2;
        if (d3 > l_d) l_d = d3;
    }
    fclose(f);
    int U = nel - j;
    if (s) {
        s->U = U;
        s->X = calloc(6 * (size_t)U, sizeof(double));
        s->region = calloc(U, sizeof(int));
        s->neig = calloc(3 * (size_t)U, sizeof(int));
        s->fneig = calloc(3 * (size_t)U, sizeof(int));
        s->dir = calloc(3 * (size_t)U, sizeof(int));
        for (int i = j + 1; i <= nel; ++i) {   /* meshList(i-j) = meshList2(i) */
            int e = i - j - 1;
            s->region[e] = reg[i];
            for (int k = 0; k < 3; ++k) {
                s->X[6 * e + 2 * k] = vx[xp[i][k]];
                s->X[6 * e + 2 * k + 1] = vy[xp[i][k]];
            }
        }
        for (int a = 1; a <= U; ++a) {
            int no_neig = 0;
            for (int b = a + 1; b <= U; ++b) {
                check_neig(s, a, b, &no_neig, l_d);
                if (no_neig == 3) break;
            }
        }
        /* transport_tri_semi.F90:222-228 + Msh2Tri.F90:463-468 getNeigDataMesh: fNeig = NumLoc(Neig(Npos), Mpos) */
        for (int e = 0; e < U; ++e)
            for (int fc = 0; fc < 3; ++fc) {
                int np = s->neig[3 * e + fc], ns = 0;
                if (np != 0) {
                    for (int q = 0; q < 3; ++q) if (s->neig[3 * (np - 1) + q] == e + 1) { ns = q + 1; break; }
                }
                s->fneig[3 * e + fc] = ns;
            }
    }
    free(vx); free(vy); free(pos_of); free(reg); free(xp);
    return U;
}

/* ------------------------------------------------------- geometry/stencils */

static const double N_gl[NGI][NLOC] = {{0.5, 0.5, 0.0}, {0.0, 0.5, 0.5}, {0.5, 0.0, 0.5}};  /* TRIQUAold :554-563, SHATRIold :1036-1040 */
static const double NLX[2][NLOC] = {{1.0, 0.0, -1.0}, {0.0, 1.0, -1.0}};                    /* SHATRIold :1042-1048 */

/* ShapFun.F90:1389-1454 tri_det_nlx + :1678-1683 per-level scaling */
static void level_geometry(const double *X, int i_split, double detwei[NGI], double nx[NGI][2][NLOC]) {
    const double weight = 1.0 / 3.0;
    for (int g = 0; g < NGI; ++g) {
        double agi = 0, bgi = 0, cgi = 0, dgi = 0;
        for (int L = 0; L < NLOC; ++L) {
            agi = agi + NLX[0][L] * X[2 * L];
            bgi = bgi + NLX[0][L] * X[2 * L + 1];
            cgi = cgi + NLX[1][L] * X[2 * L];
            dgi = dgi + NLX[1][L] * X[2 * L + 1];
        }
        double detj = agi * dgi - bgi * cgi;
        detwei[g] = 0.5 * fabs(detj) * weight;
        double a11 = dgi / detj, a21 = -(cgi / detj), a12 = -(bgi / detj), a22 = agi / detj;
        for (int L = 0; L < NLOC; ++L) {
            nx[g][0][L] = a11 * NLX[0][L] + a12 * NLX[1][L];
            nx[g][1][L] = a21 * NLX[0][L] + a22 * NLX[1][L];
        }
        detwei[g] = detwei[g] / (double)(1 << (2 * i_split));
        for (int d = 0; d < 2; ++d)
            for (int L = 0; L < NLOC; ++L) nx[g][d][L] = nx[g][d][L] * (double)(1 << i_split);
    }
}

/* ShapFun_unstruc.F90:304-335 + transport_tri_semi.F90:602-606 (diff_vol1 reduction) */
static void stencil(const double detwei[NGI], double nx[NGI][2][NLOC], double k,
                    double M[3][3], double Kd[3][3], double ml[3]) {
    for (int j = 0; j < NLOC; ++j) {
        double s = 0;
        for (int g = 0; g < NGI; ++g) s = s + N_gl[g][j] * detwei[g];
        ml[j] = s;
        for (int i = 0; i < NLOC; ++i) {
            double m = 0;
            for (int g = 0; g < NGI; ++g) m = m + N_gl[g][i] * detwei[g] * N_gl[g][j];
            M[i][j] = m;
        }
    }
    for (int i = 0; i < NLOC; ++i)
        for (int j = 0; j < NLOC; ++j) {
            double acc = 0.0;
            for (int d = 0; d < 2; ++d) {
                double s = 0;
                for (int g = 0; g < NGI; ++g) s = s + k * nx[g][d][i] * detwei[g] * nx[g][d][j];
                acc = acc + s;
            }
            Kd[i][j] = acc;
        }
}

/* ------------------------------------------------------------ the state */

static size_t lvl_len(orc_state *s, int l) { return (size_t)3 * s->nsub[l - 1] * s->U; }

static void copy_to_tnn(orc_state *s, int l) {   /* :325-327 realloc + copy */
    free(s->tnn);
    s->tnn = malloc(lvl_len(s, l) * sizeof(double));
    memcpy(s->tnn, s->tnew[l - 1], lvl_len(s, l) * sizeof(double));
    s->tnn_level = l;
}

/* splitting.F90:1210-1397 update_overlaps (faces in the order 1, 3, 2) */
static void update_overlaps(orc_state *s, int l) {
    int i_split = s->c.n_split - l + 1, m = 1 << i_split, sl = s->slots;
    int *surf = malloc(sizeof(int) * 3 * m);
    loc_surf_ele(i_split, surf);
    const double *T = s->tnew[l - 1], *To = s->told[l - 1];
    int nsub = s->nsub[l - 1];
    static const int face_order[3] = {1, 3, 2};
    PAMG_ORC_PARALLEL
    for (int u = 0; u < s->U; ++u) {
        for (int fo = 0; fo < 3; ++fo) {
            int f = face_order[fo];
            for (int i = 1; i <= m; ++i) {
                int se = surf[(i - 1) + (f - 1) * m], irow = 0, ipos = 0, orient = 0;
                get_str_info(i_split, se, &irow, &ipos, &orient);
                int npos = s->neig[3 * u + f - 1];
                double xl[3][2];
                get_splitting(s->X + 6 * u, i_split, se, xl);
                const double *tv = T + (size_t)3 * ((size_t)u * nsub + se - 1);
                const double *tov = To + (size_t)3 * ((size_t)u * nsub + se - 1);
                if (npos == 0) {
                    double *ov = s->t_overlap + (size_t)u * sl * 3 + (size_t)(f - 1) * sl;
                    double *oo = s->t_overlap_old + (size_t)u * sl * 3 + (size_t)(f - 1) * sl;
                    int a, b, na, nb;   /* 1-based slots and local nodes */
                    if (f == 1) { a = (ipos / 2) * 3 + 1; b = (ipos / 2) * 3 + 3; na = 0; nb = 2; }
                    else if (f == 3) { a = (irow - 1) * 3 + 2; b = (irow - 1) * 3 + 3; na = 1; nb = 2; }
                    else { a = (irow - 1) * 3 + 1; b = (irow - 1) * 3 + 2; na = 0; nb = 1; }
                    double t1 = boundary(xl[na][0], xl[na][1]), t2 = boundary(xl[nb][0], xl[nb][1]);
                    ov[a - 1] = t1; ov[b - 1] = t2; oo[a - 1] = t1; oo[b - 1] = t2;
                } else {
                    int nside = s->fneig[3 * u + f - 1], dir = s->dir[3 * u + f - 1], kslot;
                    int fwd, rev;
                    if (f == 1) { fwd = ipos / 2 + 1; rev = m - (ipos / 2 + 1) + 1; }
                    else { fwd = irow; rev = m - irow + 1; }
                    if (f == 2) { int t = fwd; fwd = rev; rev = t; }   /* face 2 is mirrored (:1354-1391) */
                    if (nside == 2) kslot = dir ? rev : fwd;
                    else kslot = dir ? fwd : rev;
                    double *ov = s->t_overlap + (size_t)(npos - 1) * sl * 3 + (size_t)(nside - 1) * sl;
                    double *oo = s->t_overlap_old + (size_t)(npos - 1) * sl * 3 + (size_t)(nside - 1) * sl;
                    for (int q = 0; q < 3; ++q) { ov[kslot * 3 - 3 + q] = tv[q]; oo[kslot * 3 - 3 + q] = tov[q]; }
                }
            }
        }
    }
    free(surf);
}

/* One sub-element visit of the smoother / residual: stencil products.
 * get_A_x :412-448 with theta, zero advection / flux / surface terms. */
static void get_A_x(const orc_state *s, const double M[3][3], const double Kd[3][3], double rdt,
                    const double *x, const double *xo, double A[3], double mo[3]) {
    double theta = s->c.theta;
    for (int i = 0; i < 3; ++i) {
        mo[i] = rdt * (M[i][0] * xo[0] + M[i][1] * xo[1] + M[i][2] * xo[2]);
        double mn = rdt * (M[i][0] * x[0] + M[i][1] * x[1] + M[i][2] * x[2]);
        double dv = Kd[i][0] * x[0] + Kd[i][1] * x[1] + Kd[i][2] * x[2];
        double sn = 0.0, fn = 0.0, ds = 0.0;
        A[i] = theta * (mn - sn + fn + dv + ds) + (1. - theta) * (mn);
    }
}

/* source (:593) + get_RHS (:452-464), level 1 only; writes rhs[3] and source */
static void get_rhs_l1(const orc_state *s, const double M[3][3], const double xl[3][2],
                       const double mo[3], double *src, double *rhs, const double *ovr) {
    double theta = s->c.theta, k = s->c.k;
    for (int i = 0; i < 3; ++i) src[i] = -(2 * k * boundary(xl[i][0], xl[i][1]));
    for (int i = 0; i < 3; ++i) {
        src[i] = ovr ? ovr[i] : M[i][0] * src[0] + M[i][1] * src[1] + M[i][2] * src[2];
        rhs[i] = theta * (mo[i] + src[i]) + (1. - theta) * (mo[i] + src[i]);
    }
}

/* The contracted operator of the build's arith = 1 (not the reference's arithmetic): the element
 * matrix A_e = rdt M + Kd formed once (pamg_setup.cpp level_stencil, kStcA), w = omega / D
 * (get_diagonal :481-486); a sweep x_i += w_i (b_i - sum_j A_ij x_j) and the residual
 * sum_j A_ij x_j - b_i as fma chains (pamg_device.h StcF). */
static void contracted_ops(const double M[3][3], const double Kd[3][3], const double ml[3], double rdt, double om,
                           double Ae[3][3], double w[3]) {
    for (int i = 0; i < 3; ++i) {
        for (int j = 0; j < 3; ++j) Ae[i][j] = rdt * M[i][j] + Kd[i][j];
        double D = rdt * ml[i] + Kd[i][i] + 0.0;
        w[i] = om / D;
    }
}

static void contracted_sweep(const double Ae[3][3], const double w[3], const double *b, double *x) {
    double t[3];
    for (int i = 0; i < 3; ++i) {
        t[i] = fma(-Ae[i][0], x[0], b[i]);
        t[i] = fma(-Ae[i][1], x[1], t[i]);
        t[i] = fma(-Ae[i][2], x[2], t[i]);
    }
    for (int i = 0; i < 3; ++i) x[i] = fma(w[i], t[i], x[i]);
}

static void contracted_residual(const double Ae[3][3], const double *x, const double *b, double *r) {
    for (int i = 0; i < 3; ++i) {
        double t = fma(Ae[i][0], x[0], -b[i]);
        t = fma(Ae[i][1], x[1], t);
        r[i] = fma(Ae[i][2], x[2], t);
    }
}

/* ---------------------------------------------- the face-coupled operator (op = 1)
 *
 * the surface terms the reference leaves commented out in its smoother
 * and residual (transport_tri_semi.F90:619-688, :789-857) -- the diffusion surface integral of
 * add_diffusion_surf (matrices.F90:66-117), (k / delta_x) int_f N_i (t - t2) ds, assembled as
 * get_diff_surf_stencl (:468-477) my_diff_surf / Neig_diff_surf, added to A x in get_A_x (:426-446)
 * and its self part to the diagonal in get_diagonal (:481-486). The reference cannot run it
 * (Mesh%S_nodes is never allocated, Structures.F90:157; the FORALL of :437-447 is a many-to-one
 * assignment), so this restatement DEFINES it, using the reference's own data:
 *  - faces of a sub-element: face_nodes F(1) = (1,3), F(2) = (3,2), F(3) = (2,1) (:142-147);
 *  - neighbour across face f inside the un_ele: str_neig(f, e) (get_str_neig_multigrid,
 *    splitting.F90:732-776); its nodes at my face nodes F1, F2 are its F2, F1 (the up and down
 *    sub-elements are point reflections of each other);
 *  - across an un_ele face (str_neig = 0): sp and mface as the commented loop (:626-637): f = 1 ->
 *    (ipos/2 + 1, un_ele face 1), f = 2 -> (irow, 3), f = 3 -> (irow, 2); the neighbour's three
 *    values are t_overlap(3sp-2 : 3sp, mface), written by update_overlaps (splitting.F90:1210-1397)
 *    -- its slot geometry checked against the coordinates (scripts in DESIGN.md 7) -- and
 *    S_nodes, which of them sit at my face nodes, is derived from the coordinates here; at a
 *    domain boundary the slot holds the boundary values sin(x + y) at my own face nodes;
 *  - face matrix: the P1 edge mass matrix |e| / 6 [[2, 1], [1, 2]] (the 2-point rule of the
 *    reference's face shape functions integrates it exactly) times k / delta_x, delta_x the
 *    distance between the two sub-elements' centroids (between the centroid and the face
 *    midpoint at a domain boundary, add_diffusion_surf's :90-104);
 *  - smoothing: the block (3x3) smoother of the reference with the face terms, as red-black
 *    Gauss-Seidel -- up sub-elements, then down ones (every inner neighbour of an up sub-element
 *    is a down one) -- for solver 3, Jacobi for solver 1; the values across un_ele faces are
 *    the halo snapshot update_overlaps takes at the start of every sweep (:555);
 *  - get_residual refreshes the halo from tnew first, so res = A tnew - RHS is consistent. */
static const int FNODE[3][2] = {{1, 3}, {3, 2}, {2, 1}};
static const int FMFACE[3] = {1, 3, 2};

/* splitting.F90:732-776 get_str_neig_multigrid: sn[(f - 1) + 3 (e - 1)] */
static void get_str_neig(int n, int *sn) {
    int total = (1 << (n + 1)) - 1, current = total, irow = (1 << n) - 1, ele;
#define SN(f, e) sn[((f) - 1) + 3 * ((e) - 1)]
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
#undef SN
}

static double dist2d(const double a[2], const double b[2]) {
    double dx = a[0] - b[0], dy = a[1] - b[1];
    return sqrt(dx * dx + dy * dy);
}

static void centroid(double xl[3][2], double c[2]) {
    for (int d = 0; d < 2; ++d) c[d] = (xl[0][d] + xl[1][d] + xl[2][d]) / 3.0;
}

/* face weight k / delta_x * |e| / 6 */
static double face_weight(double k, double delta, double len) { return k / delta * len / 6.0; }

/* slot that update_overlaps gives the sub-element at position i of face f of un_ele q (splitting.F90:1297-1391) */
static int overlap_kslot(const orc_state *s, int q, int f, int i_split, int i) {
    int m = 1 << i_split, *surf = malloc(sizeof(int) * 3 * m), irow = 0, ipos = 0, orient = 0, fwd, rev;
    loc_surf_ele(i_split, surf);
    get_str_info(i_split, surf[(i - 1) + (f - 1) * m], &irow, &ipos, &orient);
    free(surf);
    if (f == 1) { fwd = ipos / 2 + 1; rev = m - (ipos / 2 + 1) + 1; }
    else { fwd = irow; rev = m - irow + 1; }
    if (f == 2) { int t = fwd; fwd = rev; rev = t; }
    int nside = s->fneig[3 * q + f - 1], dr = s->dir[3 * q + f - 1];
    return (nside == 2) ? (dr ? rev : fwd) : (dr ? fwd : rev);
}

static int face_setup(orc_state *s) {
    double rdt = 1 / s->c.dt;
    for (int l = 1; l <= s->c.levels; ++l) {
        int is = s->c.n_split - l + 1, nsub = s->nsub[l - 1], m = 1 << is;
        int *sn = malloc(sizeof(int) * 3 * nsub), *surf = malloc(sizeof(int) * 3 * m);
        get_str_neig(is, sn);
        loc_surf_ele(is, surf);
        s->fnb[l - 1] = malloc(sizeof(int) * 3 * nsub);
        s->fw[l - 1] = calloc((size_t)9 * s->U, sizeof(double));
        s->fsx[l - 1] = calloc((size_t)3 * s->U, sizeof(int));
        for (int e = 1; e <= nsub; ++e) {
            int irow = 0, ipos = 0, orient = 0;
            get_str_info(is, e, &irow, &ipos, &orient);
            for (int f = 1; f <= 3; ++f) {
                int nb = sn[(f - 1) + 3 * (e - 1)];
                int sp = (f == 1) ? ipos / 2 + 1 : irow;
                s->fnb[l - 1][(f - 1) + 3 * (e - 1)] = nb ? nb : -sp;
            }
        }
        for (int u = 0; u < s->U; ++u) {
            const double *X = s->X + 6 * u;
            double *w = s->fw[l - 1] + 9 * u;
            /* inner faces: the first up sub-element (str_ele order) with a neighbour across f */
            for (int f = 1; f <= 3; ++f) {
                for (int e = 1; e <= nsub; ++e) {
                    int irow = 0, ipos = 0, orient = 0, nb = sn[(f - 1) + 3 * (e - 1)];
                    get_str_info(is, e, &irow, &ipos, &orient);
                    if (!(ipos % 2) || !nb) continue;
                    double xe[3][2], xn[3][2], ce[2], cn[2];
                    get_splitting(X, is, e, xe);
                    get_splitting(X, is, nb, xn);
                    centroid(xe, ce);
                    centroid(xn, cn);
                    w[f - 1] = face_weight(s->c.k, dist2d(ce, cn), dist2d(xe[FNODE[f - 1][0] - 1], xe[FNODE[f - 1][1] - 1]));
                    break;
                }
            }
            /* un_ele faces: the boundary sub-element at sp = 1 and what faces it */
            for (int fi = 0; fi < 3; ++fi) {
                int mface = FMFACE[fi], se = surf[0 + (mface - 1) * m];
                int a = FNODE[fi][0], b = FNODE[fi][1];
                double xe[3][2], ce[2];
                get_splitting(X, is, se, xe);
                centroid(xe, ce);
                double len = dist2d(xe[a - 1], xe[b - 1]);
                int npos = s->neig[3 * u + mface - 1];
                if (npos == 0) {
                    double mid[2] = {(xe[a - 1][0] + xe[b - 1][0]) / 2.0, (xe[a - 1][1] + xe[b - 1][1]) / 2.0};
                    w[3 + mface - 1] = face_weight(s->c.k, dist2d(ce, mid), len);
                    s->fsx[l - 1][3 * u + mface - 1] = a | (b << 2);
                    continue;
                }
                int q = npos - 1, nside = s->fneig[3 * u + mface - 1], found = 0;
                for (int i = 1; i <= m && !found; ++i) {
                    if (overlap_kslot(s, q, nside, is, i) != 1) continue;
                    double xn[3][2], cn[2];
                    get_splitting(s->X + 6 * q, is, surf[(i - 1) + (nside - 1) * m], xn);
                    centroid(xn, cn);
                    int S[2] = {0, 0};
                    for (int t = 0; t < 2; ++t) {
                        const double *p = xe[(t ? b : a) - 1];
                        double best = 1e300;
                        for (int r = 0; r < 3; ++r) {
                            double d = dist2d(p, xn[r]);
                            if (d < best) { best = d; S[t] = r + 1; }
                        }
                        if (best > 1e-9 * len) { free(sn); free(surf); return -1; }   /* slot geometry broken */
                    }
                    w[3 + mface - 1] = face_weight(s->c.k, dist2d(ce, cn), len);
                    s->fsx[l - 1][3 * u + mface - 1] = S[0] | (S[1] << 2);
                    found = 1;
                }
                if (!found) { free(sn); free(surf); return -2; }
            }
            /* D0 = rdt ml + Kd_ii + 0.0 (get_diagonal :481-486) */
            double M[3][3], Kd[3][3], ml[3];
            stencil(s->detwei[l - 1] + 3 * u, (double (*)[2][NLOC])(s->nx[l - 1] + 18 * (size_t)u), s->c.k, M, Kd, ml);
            for (int i = 0; i < 3; ++i) w[6 + i] = rdt * ml[i] + Kd[i][i] + 0.0;
        }
        free(sn);
        free(surf);
    }
    return 0;
}

/* the face terms of sub-element e (0-based index o = 3 (u nsub + e - 1)) and its diagonal:
 * ds_i = sum_{f ∋ i} w_f ((2 x_i + x_j) - 2 y_i - y_j) (faces in order), D_i = D0_i + sum_{f ∋ i} 2 w_f;
 * y = the neighbour's values at my face nodes: inner ones from `src` (the level's array the
 * neighbour's iterate is read from), across an un_ele face from t_overlap */
static void face_terms(const orc_state *s, int l, int u, int e, const double *x, const double *src, double ds[3],
                       double D[3]) {
    int nsub = s->nsub[l - 1], sl = s->slots;
    const double *w = s->fw[l - 1] + 9 * u;
    for (int i = 0; i < 3; ++i) { ds[i] = 0.0; D[i] = w[6 + i]; }
    for (int fi = 0; fi < 3; ++fi) {
        int a = FNODE[fi][0] - 1, b = FNODE[fi][1] - 1, nb = s->fnb[l - 1][fi + 3 * (e - 1)];
        double ya, yb, wf;
        if (nb > 0) {
            const double *yn = src + (size_t)3 * ((size_t)u * nsub + nb - 1);
            ya = yn[b];
            yb = yn[a];
            wf = w[fi];
        } else {
            int mface = FMFACE[fi], sx = s->fsx[l - 1][3 * u + mface - 1];
            const double *slot = s->t_overlap + (size_t)u * sl * 3 + (size_t)(mface - 1) * sl + (size_t)(-nb - 1) * 3;
            if (l > 1 && s->neig[3 * u + mface - 1] == 0) {
                ya = 0.0;   /* the coarse levels carry the error equation: homogeneous boundary data */
                yb = 0.0;
            } else {
                ya = slot[(sx & 3) - 1];
                yb = slot[((sx >> 2) & 3) - 1];
            }
            wf = w[3 + mface - 1];
        }
        ds[a] = ds[a] + wf * (((2.0 * x[a] + x[b]) - 2.0 * ya) - yb);
        ds[b] = ds[b] + wf * (((x[a] + 2.0 * x[b]) - ya) - 2.0 * yb);
        D[a] = D[a] + 2.0 * wf;
        D[b] = D[b] + 2.0 * wf;
    }
}

/* one smoother sweep of the face-coupled operator after the halo snapshot: solver 3 red-black
 * (up sub-elements from tnn, then down ones, in place), solver 1 Jacobi (from tnew, the sweep's
 * start) */
static void face_sweep(orc_state *s, int l) {
    int nsub = s->nsub[l - 1], i_split = s->c.n_split - l + 1;
    double rdt = 1 / s->c.dt, om = s->c.omega;
    double *T = s->tnew[l - 1], *To = s->told[l - 1], *R = s->rhs[l - 1], *Src = s->source[l - 1];
    for (int color = 1; color >= 0; --color) {
        PAMG_ORC_PARALLEL
        for (int u = 0; u < s->U; ++u) {
            double M[3][3], Kd[3][3], ml[3];
            stencil(s->detwei[l - 1] + 3 * u, (double (*)[2][NLOC])(s->nx[l - 1] + 18 * (size_t)u), s->c.k, M, Kd, ml);
            for (int se = 1; se <= nsub; ++se) {
                int irow = 0, ipos = 0, orient = 0;
                get_str_info(i_split, se, &irow, &ipos, &orient);
                if (s->c.solver == 3 && (ipos % 2) != color) continue;
                if (s->c.solver != 3 && color == 0) continue;   /* Jacobi: one pass */
                size_t o = (size_t)3 * ((size_t)u * nsub + se - 1);
                double xl[3][2], A[3], mo[3], ds[3], D[3];
                get_splitting(s->X + 6 * u, i_split, se, xl);
                const double *xin = (s->c.solver == 3) ? s->tnn + o : T + o;
                get_A_x(s, M, Kd, rdt, xin, To + o, A, mo);
                if (l == 1) get_rhs_l1(s, M, xl, mo, Src + o, R + o, s->src_override ? s->src_override + o : NULL);
                face_terms(s, l, u, se, xin, (s->c.solver == 3) ? s->tnn : T, ds, D);
                double x[3] = {xin[0], xin[1], xin[2]};
                for (int i = 0; i < 3; ++i) A[i] = A[i] + ds[i];
                for (int i = 0; i < 3; ++i) s->tnn[o + i] = x[i] + om / D[i] * (R[o + i] - A[i]);
            }
        }
    }
}

/* res = A tnew - RHS (neg: RHS - A tnew) of the face-coupled operator, halo refreshed from tnew */
static void face_residual(orc_state *s, int l, int neg) {
    int nsub = s->nsub[l - 1], i_split = s->c.n_split - l + 1;
    double rdt = 1 / s->c.dt;
    double *T = s->tnew[l - 1], *To = s->told[l - 1], *R = s->rhs[l - 1], *Src = s->source[l - 1];
    update_overlaps(s, l);
    PAMG_ORC_PARALLEL
    for (int u = 0; u < s->U; ++u) {
        double M[3][3], Kd[3][3], ml[3];
        stencil(s->detwei[l - 1] + 3 * u, (double (*)[2][NLOC])(s->nx[l - 1] + 18 * (size_t)u), s->c.k, M, Kd, ml);
        for (int se = 1; se <= nsub; ++se) {
            size_t o = (size_t)3 * ((size_t)u * nsub + se - 1);
            double xl[3][2], A[3], mo[3], ds[3], D[3];
            get_splitting(s->X + 6 * u, i_split, se, xl);
            get_A_x(s, M, Kd, rdt, T + o, To + o, A, mo);
            if (l == 1) get_rhs_l1(s, M, xl, mo, Src + o, R + o, s->src_override ? s->src_override + o : NULL);
            face_terms(s, l, u, se, T + o, T, ds, D);
            for (int i = 0; i < 3; ++i) {
                double a = A[i] + ds[i];
                s->res[l - 1][o + i] = neg ? R[o + i] - a : a - R[o + i];
            }
        }
    }
}

/* transport_tri_semi.F90:543-722 smoother */
static void smoother(orc_state *s, int l) {
    int i_split = s->c.n_split - l + 1, nsub = s->nsub[l - 1];
    double rdt = 1 / s->c.dt, om = s->c.omega;
    double *T = s->tnew[l - 1], *To = s->told[l - 1], *R = s->rhs[l - 1], *Src = s->source[l - 1];
    for (int sm = 0; sm < s->c.n_smooth; ++sm) {
        memcpy(T, s->tnn, lvl_len(s, l) * sizeof(double));     /* :550 */
        update_overlaps(s, l);                                  /* :555 */
        if (s->c.op == 1) {
            face_sweep(s, l);
            continue;
        }
        PAMG_ORC_PARALLEL
        for (int u = 0; u < s->U; ++u) {
            double M[3][3], Kd[3][3], ml[3];
            stencil(s->detwei[l - 1] + 3 * u, (double (*)[2][NLOC])(s->nx[l - 1] + 18 * (size_t)u), s->c.k, M, Kd, ml);
            for (int se = 1; se <= nsub; ++se) {
                size_t o = (size_t)3 * ((size_t)u * nsub + se - 1);
                double xl[3][2];
                get_splitting(s->X + 6 * u, i_split, se, xl);
                double *tnn = s->tnn + o;
                if (s->c.solver == 2) {   /* solve_Richardson :511-518, mass/stiff/flux reset to 0 at :585-612 */
                    for (int i = 0; i < 3; ++i) Src[o + i] = -(2 * s->c.k * boundary(xl[i][0], xl[i][1]));
                    for (int i = 0; i < 3; ++i) tnn[i] = tnn[i] + om * (R[o + i] - (0.0 - 0.0 + 0.0));
                    continue;
                }
                double A[3], mo[3], D[3];
                const double *xin = (s->c.solver == 3) ? tnn : T + o;   /* get_A_x(.true./.false.) */
                get_A_x(s, M, Kd, rdt, xin, To + o, A, mo);
                if (l == 1) get_rhs_l1(s, M, xl, mo, Src + o, R + o, s->src_override ? s->src_override + o : NULL);
                else for (int i = 0; i < 3; ++i) Src[o + i] = -(2 * s->c.k * boundary(xl[i][0], xl[i][1]));
                if (s->c.arith == 1) {   /* the build's contracted arithmetic (Jacobi = GS here) */
                    double Ae[3][3], w[3], x[3];
                    contracted_ops(M, Kd, ml, rdt, om, Ae, w);
                    for (int i = 0; i < 3; ++i) x[i] = xin[i];
                    contracted_sweep(Ae, w, R + o, x);
                    for (int i = 0; i < 3; ++i) tnn[i] = x[i];
                    continue;
                }
                for (int i = 0; i < 3; ++i) D[i] = rdt * ml[i] + Kd[i][i] + 0.0;   /* get_diagonal :481-486 */
                for (int i = 0; i < 3; ++i) {
                    double base = (s->c.solver == 3) ? tnn[i] : T[o + i];   /* :504 vs :494 */
                    tnn[i] = base + om / D[i] * (R[o + i] - A[i]);
                }
            }
        }
    }
}

/* transport_tri_semi.F90:725-873 get_residual */
static void get_residual(orc_state *s, int l) {
    if (s->c.op == 1) {
        face_residual(s, l, 0);
        return;
    }
    int i_split = s->c.n_split - l + 1, nsub = s->nsub[l - 1];
    double rdt = 1 / s->c.dt;
    double *T = s->tnew[l - 1], *To = s->told[l - 1], *R = s->rhs[l - 1], *Src = s->source[l - 1];
    PAMG_ORC_PARALLEL
    for (int u = 0; u < s->U; ++u) {
        double M[3][3], Kd[3][3], ml[3];
        stencil(s->detwei[l - 1] + 3 * u, (double (*)[2][NLOC])(s->nx[l - 1] + 18 * (size_t)u), s->c.k, M, Kd, ml);
        for (int se = 1; se <= nsub; ++se) {
            size_t o = (size_t)3 * ((size_t)u * nsub + se - 1);
            double xl[3][2], A[3], mo[3];
            get_splitting(s->X + 6 * u, i_split, se, xl);
            get_A_x(s, M, Kd, rdt, T + o, To + o, A, mo);
            if (l == 1) get_rhs_l1(s, M, xl, mo, Src + o, R + o, s->src_override ? s->src_override + o : NULL);
            else for (int i = 0; i < 3; ++i) Src[o + i] = -(2 * s->c.k * boundary(xl[i][0], xl[i][1]));
            if (s->c.arith == 1 && s->c.solver != 2) {
                double Ae[3][3], w[3];
                contracted_ops(M, Kd, ml, rdt, s->c.omega, Ae, w);
                contracted_residual(Ae, T + o, R + o, s->res[l - 1] + o);
                continue;
            }
            for (int i = 0; i < 3; ++i) s->res[l - 1][o + i] = A[i] - R[o + i];
        }
    }
}

/* splitting.F90:10-32 restrictor */
static void restrictor(orc_state *s, int l) {
    if (l >= s->c.levels) return;
    int i_split = s->c.n_split - l + 1, nf = s->nsub[l - 1], nc = s->nsub[l];
    const double *r = s->res[l - 1];
    double *b = s->rhs[l];
    PAMG_ORC_PARALLEL
    for (int u = 0; u < s->U; ++u)
        for (int c = 1; c <= nc; ++c) {
            int fin[4];
            element_conversion(fin, c, i_split - 1);
            const int pick[3] = {fin[2], fin[3], fin[0]};
            for (int i = 0; i < 3; ++i) {
                const double *rv = r + (size_t)3 * ((size_t)u * nf + pick[i] - 1);
                b[(size_t)3 * ((size_t)u * nc + c - 1) + i] = (rv[0] + rv[1] + rv[2]) / 3.;
            }
        }
}

/* splitting.F90:38-91 prolongator */
static void prolongator(orc_state *s, int l) {
    int i_split = s->c.n_split - l + 1, nf = s->nsub[l - 1], nc = s->nsub[l];
    double *F = s->tnew[l - 1];
    const double *Y = s->tnew[l];
    PAMG_ORC_PARALLEL
    for (int u = 0; u < s->U; ++u)
        for (int c = 1; c <= nc; ++c) {
            int fin[4];
            element_conversion(fin, c, i_split - 1);
            const double *y = Y + (size_t)3 * ((size_t)u * nc + c - 1);
            double *f1 = F + (size_t)3 * ((size_t)u * nf + fin[0] - 1);
            double *f2 = F + (size_t)3 * ((size_t)u * nf + fin[1] - 1);
            double *f3 = F + (size_t)3 * ((size_t)u * nf + fin[2] - 1);
            double *f4 = F + (size_t)3 * ((size_t)u * nf + fin[3] - 1);
            f1[0] = f1[0] + 0.5 * y[2] + 0.5 * y[0];
            f1[1] = f1[1] + 0.5 * y[1] + 0.5 * y[2];
            f1[2] = f1[2] + y[2];
            f2[0] = f2[0] + f1[1];
            f2[1] = f2[1] + f1[0];
            f2[2] = f2[2] + 0.5 * y[0] + 0.5 * y[1];
            f3[0] = f3[0] + y[0];
            f3[1] = f3[1] + f2[2];
            f3[2] = f3[2] + f2[1];
            f4[0] = f4[0] + f2[2];
            f4[1] = f4[1] + y[1];
            f4[2] = f4[2] + f2[0];
        }
}

/* matrix_inversion.F90:50-148 FINDInv: Gauss-Jordan on the augmented matrix
 * [A | I], no pivoting; a zero pivot is repaired by adding the first lower row
 * with a nonzero entry in that column (:75-86) -- but the search gives up at the
 * first zero entry (:87-92); matrices are column-major (n, n). Returns the
 * errorflag (0 / -1; inverse = 0 on -1). */
int orc_findinv(int n, const double *A, double *inv) {
    double aug[16][32];
    if (n < 1 || n > 16) return -2;
#define AG(i, j) aug[(i) - 1][(j) - 1]
    for (int i = 1; i <= n; ++i)
        for (int j = 1; j <= 2 * n; ++j) {
            if (j <= n) AG(i, j) = A[(i - 1) + (size_t)(j - 1) * n];
            else if (i + n == j) AG(i, j) = 1;
            else AG(i, j) = 0;
        }
    for (int k = 1; k <= n - 1; ++k) {
        if (AG(k, k) == 0) {
            int flag = 0;
            for (int i = k + 1; i <= n; ++i) {
                if (AG(i, k) != 0) {
                    for (int j = 1; j <= 2 * n; ++j) AG(k, j) = AG(k, j) + AG(i, j);
                    flag = 1;
                    break;
                }
                if (!flag) {
                    for (int q = 0; q < n * n; ++q) inv[q] = 0;
                    return -1;
                }
            }
        }
        for (int j = k + 1; j <= n; ++j) {
            double m = AG(j, k) / AG(k, k);
            for (int i = k; i <= 2 * n; ++i) AG(j, i) = AG(j, i) - m * AG(k, i);
        }
    }
    for (int i = 1; i <= n; ++i)
        if (AG(i, i) == 0) {
            for (int q = 0; q < n * n; ++q) inv[q] = 0;
            return -1;
        }
    for (int i = 1; i <= n; ++i) {
        double m = AG(i, i);
        for (int j = i; j <= 2 * n; ++j) AG(i, j) = AG(i, j) / m;
    }
    for (int k = n - 1; k >= 1; --k)
        for (int i = 1; i <= k; ++i) {
            double m = AG(i, k + 1);
            for (int j = k; j <= 2 * n; ++j) AG(i, j) = AG(i, j) - AG(k + 1, j) * m;
        }
    for (int i = 1; i <= n; ++i)
        for (int j = 1; j <= n; ++j) inv[(i - 1) + (size_t)(j - 1) * n] = AG(i, j + n);
#undef AG
    return 0;
}

/* THE BUILD'S DIRECT PATH (coarse_solver = 1; not in the reference's mode 9):
 * tnew = tnew_nonlin = A_e^-1 RHS per sub-element, A_e = (1/dt) M + Kd the smoother's
 * operator (get_A_x :412-448 assembled, theta = 1, u = 0) inverted by FINDInv. */
static void direct_solve(orc_state *s, int l) {
    int nsub = s->nsub[l - 1];
    double rdt = 1 / s->c.dt;
    free(s->tnn);
    s->tnn = malloc(lvl_len(s, l) * sizeof(double));
    s->tnn_level = l;
    for (int u = 0; u < s->U; ++u) {
        double M[3][3], Kd[3][3], ml[3], a[9], inv[9];
        stencil(s->detwei[l - 1] + 3 * u, (double (*)[2][NLOC])(s->nx[l - 1] + 18 * (size_t)u), s->c.k, M, Kd, ml);
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) a[i + 3 * j] = rdt * M[i][j] + Kd[i][j];
        orc_findinv(3, a, inv);
        for (int se = 0; se < nsub; ++se) {
            size_t o = (size_t)3 * ((size_t)u * nsub + se);
            const double *b = s->rhs[l - 1] + o;
            for (int i = 0; i < 3; ++i) {
                double x = inv[i] * b[0] + inv[i + 3] * b[1] + inv[i + 6] * b[2];
                s->tnew[l - 1][o + i] = x;
                s->tnn[o + i] = x;
            }
        }
    }
}

/* ----------------------------------------------------------- public API */

int orc_msh_count(const char *path) { return read_msh(path, NULL); }

/* Mesh + topology exactly as the reference builds it (ReadMSH/CheckNeig/getNeigDataMesh). */
int orc_msh_load(const char *path, int U, double *X, int *region, int *neig, int *fneig, int *dir) {
    orc_state s;
    memset(&s, 0, sizeof s);
    int n = read_msh(path, &s);
    if (n < 0) return n;
    if (n != U) return -10;
    memcpy(X, s.X, sizeof(double) * 6 * U);
    memcpy(region, s.region, sizeof(int) * U);
    memcpy(neig, s.neig, sizeof(int) * 3 * U);
    memcpy(fneig, s.fneig, sizeof(int) * 3 * U);
    memcpy(dir, s.dir, sizeof(int) * 3 * U);
    free(s.X); free(s.region); free(s.neig); free(s.fneig); free(s.dir);
    return 0;
}

void orc_free(orc_state *s);

orc_state *orc_create(const orc_cfg *cfg, int U, const double *X, const int *region, const int *neig,
                      const int *fneig, const int *dir) {
    if (cfg->levels < 1 || cfg->levels > cfg->n_split || cfg->n_split > 12) return NULL;  /* :120-123 */
    if (cfg->theta != 1.0) return NULL;   /* theta hard-coded to 1 (:117); the theta<1 RHS is iterate-dependent */
    orc_state *s = calloc(1, sizeof *s);
    s->c = *cfg;
    s->U = U;
    s->X = malloc(sizeof(double) * 6 * U); memcpy(s->X, X, sizeof(double) * 6 * U);
    s->region = malloc(sizeof(int) * U); memcpy(s->region, region, sizeof(int) * U);
    s->neig = malloc(sizeof(int) * 3 * U); memcpy(s->neig, neig, sizeof(int) * 3 * U);
    s->fneig = malloc(sizeof(int) * 3 * U); memcpy(s->fneig, fneig, sizeof(int) * 3 * U);
    s->dir = malloc(sizeof(int) * 3 * U); memcpy(s->dir, dir, sizeof(int) * 3 * U);
    for (int l = 1; l <= cfg->levels; ++l) {
        int i_split = cfg->n_split - l + 1;
        s->nsub[l - 1] = 1 << (2 * i_split);
        size_t n = lvl_len(s, l);
        s->tnew[l - 1] = calloc(n, sizeof(double));
        s->told[l - 1] = calloc(n, sizeof(double));
        s->rhs[l - 1] = calloc(n, sizeof(double));
        s->res[l - 1] = calloc(n, sizeof(double));
        s->source[l - 1] = calloc(n, sizeof(double));
        s->detwei[l - 1] = calloc((size_t)3 * U, sizeof(double));
        s->nx[l - 1] = calloc((size_t)18 * U, sizeof(double));
        for (int u = 0; u < U; ++u)
            level_geometry(s->X + 6 * u, i_split, s->detwei[l - 1] + 3 * u,
                           (double (*)[2][NLOC])(s->nx[l - 1] + 18 * (size_t)u));
    }
    /* :249-251 region 4 => tnew(level 1) = 1 */
    for (int u = 0; u < U; ++u)
        if (s->region[u] == 4)
            for (int q = 0; q < 3 * s->nsub[0]; ++q) s->tnew[0][(size_t)3 * s->nsub[0] * u + q] = 1.0;
    s->slots = (1 << cfg->n_split) * 3;
    s->t_overlap = calloc((size_t)s->slots * 3 * U, sizeof(double));
    s->t_overlap_old = calloc((size_t)s->slots * 3 * U, sizeof(double));
    copy_to_tnn(s, 1);
    if (cfg->op == 1 && (cfg->solver == 2 || cfg->coarse_solver == 1 || face_setup(s) != 0)) {
        orc_free(s);
        return NULL;
    }
    return s;
}

void orc_free(orc_state *s) {
    if (!s) return;
    for (int l = 0; l < s->c.levels; ++l) {
        free(s->tnew[l]); free(s->told[l]); free(s->rhs[l]); free(s->res[l]); free(s->source[l]);
        free(s->detwei[l]); free(s->nx[l]);
        free(s->fnb[l]); free(s->fw[l]); free(s->fsx[l]);
    }
    free(s->tnn); free(s->t_overlap); free(s->t_overlap_old); free(s->src_override);
    free(s->X); free(s->region); free(s->neig); free(s->fneig); free(s->dir);
    free(s);
}

/* what: 0 tnew, 1 told, 2 rhs, 3 res, 4 tnn (level ignored), 5 source */
static double *field(orc_state *s, int what, int l, size_t *n) {
    if (what == 4) { *n = lvl_len(s, s->tnn_level); return s->tnn; }
    if (l < 1 || l > s->c.levels) return NULL;
    *n = lvl_len(s, l);
    switch (what) {
        case 0: return s->tnew[l - 1];
        case 1: return s->told[l - 1];
        case 2: return s->rhs[l - 1];
        case 3: return s->res[l - 1];
        case 5: return s->source[l - 1];
    }
    return NULL;
}

long orc_get(orc_state *s, int what, int l, double *out) {
    size_t n; double *p = field(s, what, l, &n);
    if (!p) return -1;
    if (out) memcpy(out, p, n * sizeof(double));
    return (long)n;
}

int orc_set(orc_state *s, int what, int l, const double *in) {
    size_t n; double *p = field(s, what, l, &n);
    if (!p) return -1;
    memcpy(p, in, n * sizeof(double));
    return 0;
}

int orc_tnn_level(orc_state *s) { return s->tnn_level; }

/* test hook: level 1's cascaded source term s' in the (3, nsub_1, U) layout (NULL: evaluate it) */
int orc_set_source(orc_state *s, const double *src1) {
    free(s->src_override);
    s->src_override = NULL;
    if (!src1) return 0;
    s->src_override = malloc(lvl_len(s, 1) * sizeof(double));
    if (!s->src_override) return -1;
    memcpy(s->src_override, src1, lvl_len(s, 1) * sizeof(double));
    return 0;
}

void orc_get_overlap(orc_state *s, double *tov, double *tovo) {
    size_t n = (size_t)s->slots * 3 * s->U;
    if (tov) memcpy(tov, s->t_overlap, n * sizeof(double));
    if (tovo) memcpy(tovo, s->t_overlap_old, n * sizeof(double));
}

void orc_level_geometry(orc_state *s, int l, double *detwei, double *M, double *Kd, double *ml) {
    for (int u = 0; u < s->U; ++u) {
        double m[3][3], kd[3][3], l3[3];
        stencil(s->detwei[l - 1] + 3 * u, (double (*)[2][NLOC])(s->nx[l - 1] + 18 * (size_t)u), s->c.k, m, kd, l3);
        for (int i = 0; i < 3; ++i) {
            detwei[3 * u + i] = s->detwei[l - 1][3 * u + i];
            ml[3 * u + i] = l3[i];
            for (int j = 0; j < 3; ++j) {   /* Fortran (i,j,u) column-major */
                M[9 * u + i + 3 * j] = m[i][j];
                Kd[9 * u + i + 3 * j] = kd[i][j];
            }
        }
    }
}

/* One Jacobi sweep of level l (the inner loop of the smoother, transport_tri_semi.F90:580-707,
 * solve_Jacobi :491-497 -- equal to solve_Gauss_Seidel :501-507 for this block-diagonal operator)
 * from given x and b, both (3, nsub, U) column-major: out = x + (omega / D) (b - A_e x), the
 * reference's operation order (arith 0) or the contracted one of the build's arith = 1. Nothing
 * else is touched: the checker of the level-1 roofline sweep kernels (pamg_sweep_bench_output). */
void orc_sweep_once(orc_state *s, int l, int arith, const double *x, const double *b, double *out) {
    int nsub = s->nsub[l - 1];
    double rdt = 1 / s->c.dt, om = s->c.omega;
    PAMG_ORC_PARALLEL
    for (int u = 0; u < s->U; ++u) {
        double M[3][3], Kd[3][3], ml[3], Ae[3][3], w[3], D[3];
        stencil(s->detwei[l - 1] + 3 * u, (double (*)[2][NLOC])(s->nx[l - 1] + 18 * (size_t)u), s->c.k, M, Kd, ml);
        contracted_ops(M, Kd, ml, rdt, om, Ae, w);
        for (int i = 0; i < 3; ++i) D[i] = rdt * ml[i] + Kd[i][i] + 0.0;   /* get_diagonal :481-486 */
        for (int se = 0; se < nsub; ++se) {
            size_t o = (size_t)3 * ((size_t)u * nsub + se);
            if (arith == 1) {
                double xx[3] = {x[o], x[o + 1], x[o + 2]};
                contracted_sweep(Ae, w, b + o, xx);
                for (int i = 0; i < 3; ++i) out[o + i] = xx[i];
                continue;
            }
            double A[3], mo[3];
            get_A_x(s, M, Kd, rdt, x + o, x + o, A, mo);
            for (int i = 0; i < 3; ++i) out[o + i] = x[o + i] + om / D[i] * (b[o + i] - A[i]);
        }
    }
}

void orc_copy_to_tnn(orc_state *s, int l) { copy_to_tnn(s, l); }
void orc_smoother(orc_state *s, int l) { smoother(s, l); }
void orc_get_residual(orc_state *s, int l) { get_residual(s, l); }
void orc_restrictor(orc_state *s, int l) { restrictor(s, l); }
void orc_prolongator(orc_state *s, int l) { prolongator(s, l); }
void orc_update_overlaps(orc_state *s, int l) { update_overlaps(s, l); }
void orc_direct_solve(orc_state *s, int l) { direct_solve(s, l); }

/* :316-317 */
void orc_begin_timestep(orc_state *s) {
    memcpy(s->told[0], s->tnew[0], lvl_len(s, 1) * sizeof(double));
    copy_to_tnn(s, 1);
}

/* :319-379, one pass of the n_multigrid loop (one V-cycle) */
void orc_vcycle(orc_state *s) {
    int L = s->c.levels;
    for (int l = 1; l <= L; ++l) {
        copy_to_tnn(s, l);
        smoother(s, l);
        restrictor(s, l);
        get_residual(s, l);
    }
    if (s->c.coarse_solver == 1) {
        direct_solve(s, L);
    } else {
        copy_to_tnn(s, L);
        for (int i = 0; i < s->c.n_coarse; ++i) smoother(s, L);
    }
    for (int l = L - 1; l >= 1; --l) {
        copy_to_tnn(s, l);
        prolongator(s, l);
        smoother(s, l);
    }
}

/* ---- the corrected V-cycle (the build's opt-in, no reference
 * output exists): the reference's levels, operators, smoother, restrictor weights and
 * interpolation weights, with the cycle's three defects of A3 fixed -- (iii) the
 * restrictor acts on the FRESH residual, (i)/(iv) the prolonged coarse correction is
 * added to the iterate the next smoother call starts from, and the residual has the
 * b - A x sign; coarse levels start from zero every cycle. The iterate of a level after
 * a smoother call is tnew_nonlin (the last sweep), copied to tnew. */

/* res_l = RHS_l - A_l tnew_l (get_residual's products, :725-873, with the b - A x sign) */
static void residual_corrected(orc_state *s, int l) {
    if (s->c.op == 1) {
        face_residual(s, l, 1);
        return;
    }
    int nsub = s->nsub[l - 1];
    double rdt = 1 / s->c.dt;
    double *T = s->tnew[l - 1], *To = s->told[l - 1], *R = s->rhs[l - 1];
    for (int u = 0; u < s->U; ++u) {
        double M[3][3], Kd[3][3], ml[3];
        stencil(s->detwei[l - 1] + 3 * u, (double (*)[2][NLOC])(s->nx[l - 1] + 18 * (size_t)u), s->c.k, M, Kd, ml);
        double Ae[3][3], w[3];
        if (s->c.arith == 1) contracted_ops(M, Kd, ml, rdt, s->c.omega, Ae, w);
        for (int se = 1; se <= nsub; ++se) {
            size_t o = (size_t)3 * ((size_t)u * nsub + se - 1);
            if (s->c.arith == 1) {   /* the build's contracted arithmetic: -(A x - b) of the fma rows */
                double r[3];
                contracted_residual(Ae, T + o, R + o, r);
                for (int i = 0; i < 3; ++i) s->res[l - 1][o + i] = -r[i];
                continue;
            }
            double A[3], mo[3];
            get_A_x(s, M, Kd, rdt, T + o, To + o, A, mo);
            for (int i = 0; i < 3; ++i) s->res[l - 1][o + i] = R[o + i] - A[i];
        }
    }
}

/* tnew_l += P tnew_{l+1}: the P1 interpolation the prolongator's cascade (splitting.F90:59-88)
 * encodes -- each child node gets a coarse vertex value or an edge midpoint -- applied to the
 * coarse correction alone (the cascade also feeds already-updated fine values forward) */
static void interp_add(orc_state *s, int l) {
    int i_split = s->c.n_split - l + 1, nf = s->nsub[l - 1], nc = s->nsub[l];
    double *F = s->tnew[l - 1];
    const double *Y = s->tnew[l];
    for (int u = 0; u < s->U; ++u)
        for (int c = 1; c <= nc; ++c) {
            int fin[4];
            element_conversion(fin, c, i_split - 1);
            const double *y = Y + (size_t)3 * ((size_t)u * nc + c - 1);
            const double m20 = 0.5 * y[2] + 0.5 * y[0], m12 = 0.5 * y[1] + 0.5 * y[2], m01 = 0.5 * y[0] + 0.5 * y[1];
            const double add[4][3] = {{m20, m12, y[2]}, {m12, m20, m01}, {y[0], m01, m20}, {m01, y[1], m12}};
            for (int q = 0; q < 4; ++q) {
                double *f = F + (size_t)3 * ((size_t)u * nf + fin[q] - 1);
                for (int i = 0; i < 3; ++i) f[i] = f[i] + add[q][i];
            }
        }
}

static void smooth_to_tnew(orc_state *s, int l, int calls) {
    copy_to_tnn(s, l);
    for (int i = 0; i < calls; ++i) smoother(s, l);
    memcpy(s->tnew[l - 1], s->tnn, lvl_len(s, l) * sizeof(double));
}

void orc_vcycle_corrected(orc_state *s) {
    int L = s->c.levels;
    for (int l = 1; l < L; ++l) {
        if (l > 1) memset(s->tnew[l - 1], 0, lvl_len(s, l) * sizeof(double));
        smooth_to_tnew(s, l, 1);
        residual_corrected(s, l);
        restrictor(s, l);
    }
    if (L > 1) memset(s->tnew[L - 1], 0, lvl_len(s, L) * sizeof(double));   /* a coarse level starts from zero */
    if (L == 1) {
        smooth_to_tnew(s, 1, 1);
        residual_corrected(s, 1);
    } else if (s->c.coarse_solver == 1) {
        copy_to_tnn(s, L);
        direct_solve(s, L);
    } else {
        smooth_to_tnew(s, L, s->c.n_coarse);
    }
    for (int l = L - 1; l >= 1; --l) {
        interp_add(s, l);
        smooth_to_tnew(s, l, 1);
    }
    if (L > 1) residual_corrected(s, 1);   /* the fine residual after the cycle */
}

/* :299-381 the time loop */
void orc_run(orc_state *s) {
    for (int it = 0; it < s->c.ntime; ++it) {
        orc_begin_timestep(s);
        for (int mg = 0; mg < s->c.n_multigrid; ++mg) orc_vcycle(s);
    }
}

/* matrices.F90:172-193 csr_mul_array: the entries are consumed in storage order, three per
 * row, for nrows = size(g_iloc) rows (g_iloc's values are never read); result(r) starts at
 * 0 and accumulates val(c) * array(g_jloc(c)) in that order; g_jloc is 1-based. */
void orc_csr_mul_array(long nrows, const int *g_jloc, const double *val, const double *array, double *result) {
    long c2 = 0;
    for (long r = 0; r < nrows; ++r) {
        result[r] = 0.0;
        for (int n = 0; n < 3; ++n) {
            result[r] = result[r] + val[c2] * array[g_jloc[c2] - 1];
            c2 = c2 + 1;
        }
    }
}
