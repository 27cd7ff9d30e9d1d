/*
 * pamg.h -- C-ABI of the MI355X-native multigrid hot path (libpamg.so).
 *
 * Drop-in boundary for the multigrid smoother / residual / restriction /
 * prolongation / halo loop of the reference's semi-structured DG solver
 * (Amin-Nadimy/P-A_multigrids). The reference has no FFI of its own: the path
 * is a set of internal (`contains`) subroutines of `Semi_implicit_iterative`
 * reached by host association. Each entry point below names the reference
 * routine it replaces (file:line in the reference tree). The Fortran host
 * binds these through iso_c_binding (p-a_multigrids_amd/fortran/pamg_mod.F90);
 * the Python tests / bench bind them through ctypes (p-a_multigrids_amd/pamg).
 *
 * Conventions
 *  - plain pointers and sizes only; every entry returns int (0 = PAMG_OK,
 *    < 0 = error, message via pamg_last_error); no C++ exception crosses.
 *  - host field arrays use the reference's Fortran layout
 *    tracer(l)%x(3, nsub_l, U), column-major, fp64 (Structures.F90:185-188);
 *    nsub_l = 4**(n_split - l + 1) (transport_tri_semi.F90:180).
 *  - levels are 1-based as in the reference; neighbour ids are 1-based and 0
 *    marks a domain boundary (Structures.F90:143-170 Mesh%Neig/fNeig/Dir).
 *  - device memory is owned by the handle; host copies happen only in
 *    upload / set_state / get_state / get_overlap, never per sweep.
 *  - calls are ordered on the handle's HIP stream; getters synchronise.
 */
#ifndef PAMG_H
#define PAMG_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PAMG_OK 0
#define PAMG_ERR_ARG (-1)
#define PAMG_ERR_HIP (-2)
#define PAMG_ERR_IO (-3)
#define PAMG_ERR_STATE (-4)
#define PAMG_ERR_COMM (-5)
#define PAMG_ERR_NODEV (-6)

/* field selectors for pamg_set_state / pamg_get_state (Structures.F90:185-188) */
#define PAMG_TNEW 0        /* tracer(l)%tnew */
#define PAMG_TOLD 1        /* tracer(l)%told */
#define PAMG_RHS 2         /* tracer(l)%RHS */
#define PAMG_RESIDUAL 3    /* tracer(l)%residuale */
#define PAMG_TNEW_NONLIN 4 /* tnew_nonlin (transport_tri_semi.F90:85), shape of its current level */
#define PAMG_SOURCE 5      /* tracer(1)%source after get_RHS: level 1's cascaded source term s' (:452-464,
                              :593), formed once at upload; level 1 only, pamg_get_state only */

/* timed kernel classes (pamg_timing_*) */
#define PAMG_K_SMOOTH_L1 0
#define PAMG_K_SMOOTH 1
#define PAMG_K_RESIDUAL 2
#define PAMG_K_RESTRICT 3
#define PAMG_K_PROLONG 4
#define PAMG_K_RHS 5
#define PAMG_K_HALO 6
#define PAMG_K_SWEEP_BENCH 7
#define PAMG_K_VCYCLE 8          /* fused V-cycle, level-1 launch */
#define PAMG_K_VCYCLE_COARSE 9   /* fused V-cycle, levels 2..L launch */
#define PAMG_K_VCYCLE_PIPE 10    /* pipelined fused V-cycle: level 1 of cycle c + levels 2..L of cycle c+1 */
#define PAMG_K_VCYCLE_RHSF 11    /* the pipelined launch that starts a pamg_run step (told, RHS) */
#define PAMG_K_VCYCLE_RES 12     /* resident V-cycle call: every cycle of a pamg_vcycle call in one launch */
#define PAMG_K_VCYCLE_RES_RHSF 13 /* the resident launch that starts a pamg_run step */
#define PAMG_K_VCYCLE_CORR 14    /* the corrected V-cycle's resident call (cycle = 1): a pamg_vcycle call in one launch */
#define PAMG_K_HALO_EARLY 15     /* the resident call's per-call exchange, started on a device signal once the tiles
                                    with remote faces have finished (comm stream; overlapped with the launch) */
#define PAMG_K_FACE_FALLBACK 16  /* face-operator smoother calls whose persistent chain launch found its workgroups not
                                    all resident and left the state untouched: run with one launch per sweep instead
                                    (counted in pamg_timing_issued whatever the timing mask) */
#define PAMG_K_COARSE_GATHER 17  /* op = 1 on a partition: the ranks' coarsest-level blocks (RHS each cycle, tnew once
                                    per call) gathered into every rank's replica of that level (the agglomerated
                                    coarsest level: the single-domain chain runs on each rank) */
#define PAMG_K_COUNT 18

typedef struct pamg_handle pamg_handle;
typedef struct pamg_mesh pamg_mesh;

typedef struct {
    int n_split;      /* transport_tri_semi.F90:118 */
    int multi_levels; /* main.F90:46-47 (multi_levels <= n_split, :120-123) */
    int n_smooth;     /* sweeps per smoother call, main.F90:46-47 */
    int n_coarse;     /* smoother calls on the coarsest level, :351 (15) */
    int solver;       /* 1 Jacobi, 2 Richardson, 3 Gauss-Seidel (:695-716) */
    int device;       /* HIP device ordinal */
    double dt;        /* CFL*dx, :133 */
    double k;         /* diffusion coefficient, :136 */
    double omega;     /* relaxation, :140 */
    double theta;     /* time weighting, :117 (only 1.0 is accepted) */
    int halo_mode;    /* 0: halo written once per smoother call (state-identical),
                         1: one launch per sweep, halo at every sweep (reference timing) */
    int fused;        /* default 3. 1: pamg_vcycle runs each V-cycle as two fused launches when supported
                         (solver 1/3, halo_mode 0, n_split <= 5, coarse_solver 0); 0: one kernel
                         per step; 2: the two fused launches of a cycle run concurrently on two
                         streams (the coarse levels' fp64 work under level 1's HBM stream;
                         state identical to 1); 3: pipelined -- one launch per cycle
                         runs level 1 of cycle c and the coarse levels of cycle c+1 tile by tile
                         (level 2's RHS stays in LDS; state identical to 1) */
    int coarse_solver; /* 0: the reference's n_coarse smoother calls on the coarsest level (:351-353);
                          1: its exact local solve instead, tnew = tnew_nonlin = A_e^-1 RHS with
                          A_e = (1/dt) M + Kd inverted by FINDInv (matrix_inversion.F90:50-148) --
                          the direct path of SURVEY.md 8(f), not the reference's mode 9 */
    int arith;        /* operator arithmetic of the smoother / residual kernels (solver 1/3):
                         0: the reference's operation order, no contraction -- bitwise equal to the
                            reference's fp64 build (get_A_x / solve_*, :412-507);
                         1: contracted -- A_e = (1/dt) M + Kd assembled once per un_ele (fp64, host),
                            one fma chain per row: 12 fp64 operations per sub-element sweep instead
                            of 39; within 1e-13 relative of the reference (the north star's bar
                            is 1e-10), bitwise equal between the fused and per-step schedules */
    int halo_exchange; /* multi-rank fused V-cycle: 0 (default) the RCCL exchange of the level-1 halo
                          words runs once per pamg_vcycle call, after its last cycle -- every cycle
                          rewrites every halo word and nothing in the cycle reads t_overlap, so only
                          the last cycle's words are observable (state identical to 1); 1: after
                          every cycle, overlapped with the next one */
    int cycle;        /* 0 (default): the reference's V-cycle with all its quirks;
                         1: the corrected V-cycle of SURVEY.md 8(f) rank 2 -- the restrictor acts on
                         the fresh residual b - A x, coarse levels start from zero, the prolonged
                         correction (P1 interpolation of the coarse iterate) is added to the iterate
                         the next smoother call starts from; a pamg_vcycle call runs as one resident
                         launch (every level of a tile on-chip between the cycles; op 0, coarse_solver 0,
                         fused != 0, halo_exchange 0), else as the per-step kernels -- the state is the
                         same bit for bit; no reference output exists, pinned to the oracle's restatement */
    int op;           /* 0 (default): the reference's mode-9 operator, block diagonal (its surface terms are
                         commented out, transport_tri_semi.F90:619-688); 1: the face-coupled interior-penalty
                         diffusion operator of SURVEY.md 8(f) rank 1 -- the surface terms with
                         the reference's t_overlap halo as the values across un_ele faces (read every sweep,
                         exchanged every sweep between ranks), red-black (up / down) Gauss-Seidel for
                         solver 3, Jacobi for solver 1; per-step kernels; no reference output exists (the
                         reference cannot run the block), pinned to the oracle's restatement.
                         Not with solver 2 or coarse_solver 1 */
    int reserved[1];
} pamg_params;

/* mode-9 defaults of the reference (main.F90:46-47, transport_tri_semi.F90:117-140) */
void pamg_default_params(pamg_params *p);
int pamg_version(void);

/* ---- mesh ingest: replaces ReadMSH + CheckNeig + getNeigDataMesh
 *      (Msh2Tri.F90:132-334, 776-963, 454-548) with an O(N) edge hash ---- */
int pamg_msh_read(const char *path, pamg_mesh **m);
/* structured strip of nx*ny*2 triangles on [0,lx]x[0,ly] (synthetic scaling meshes) */
int pamg_msh_strip(int nx, int ny, double lx, double ly, pamg_mesh **m);
/* gmsh 2.2 ASCII of a mesh (nodes deduplicated, coordinates to the last bit): the input format
 * of ReadMSH, so synthetic meshes feed the reference too */
int pamg_msh_write(const pamg_mesh *m, const char *path);
/* binary mesh cache (the reference re-runs its O(N^2) CheckNeig on every start,
 * grofiling.txt:6-8): X, region, Neig, fNeig, Dir with a checksum; pamg_msh_read_cached parses
 * msh_path only when cache_path is missing or was made from other file contents (FNV-1a of the
 * .msh bytes), then writes the cache; *hit = 1 when the cache was used */
int pamg_msh_save(const pamg_mesh *m, const char *path);
int pamg_msh_load(const char *path, pamg_mesh **m);
int pamg_msh_read_cached(const char *msh_path, const char *cache_path, pamg_mesh **m, int *hit);
int pamg_msh_size(const pamg_mesh *m, int *U);
/* X(2,3,U) fp64, region(U), Neig/fNeig/Dir(3,U) */
int pamg_msh_get(const pamg_mesh *m, double *X, int *region, int *neig, int *fneig, int *dir);
void pamg_msh_free(pamg_mesh *m);

/* ---- handle ---- */
int pamg_create(const pamg_params *p, pamg_handle **h);
/* mesh + topology; runs the setup of transport_tri_semi.F90:178-288 on the
 * device side (per-level stencils, numbering tables, halo plan, initial
 * condition tnew := 0, region 4 := 1 at level 1, :237-252) */
int pamg_upload_mesh(pamg_handle *h, int U, const double *X, const int *region, const int *neig,
                     const int *fneig, const int *dir);
int pamg_nsub(pamg_handle *h, int level);
int pamg_set_state(pamg_handle *h, int level, int what, const double *host);
int pamg_get_state(pamg_handle *h, int level, int what, double *host);
/* halo buffers meshList(:)%t_overlap / t_overlap_old as (2**n_split*3, 3, U) */
int pamg_get_overlap(pamg_handle *h, double *t_overlap, double *t_overlap_old);
int pamg_tnn_level(pamg_handle *h);
/* VTU of the level-1 solution: replaces get_vtu (get_vtk_files.F90:10-165, called at
 * transport_tri_semi.F90:301-311) -- the same cells (one triangle per level-1 sub-element
 * with its own 3 DG nodes) and point data ("Tracer" = tnew, "error" = |tnew - sin(x+y)|,
 * "analytical" = sin(x+y)) at full fp64 precision; ascii = 0 raw appended binary, 1 ascii.
 * Multi-rank: each rank writes its own elements (one file per rank). */
int pamg_write_vtu(pamg_handle *h, const char *path, int ascii);

/* ---- the hot path, one entry per reference call site ---- */
/* :316-317 told := tnew, tnew_nonlin := tnew, plus level-1 RHS (get_RHS :452-464) */
int pamg_begin_timestep(pamg_handle *h);
/* :325-327, :346-348, :365-367 tnew_nonlin := tracer(l)%tnew */
int pamg_copy_to_nonlin(pamg_handle *h, int level);
/* n_calls consecutive `call smoother` (:331, :352, :376; body :543-722) */
int pamg_smoother(pamg_handle *h, int level, int n_calls);
/* n_sweeps single sweeps with the smoother's tnew / tnew_nonlin semantics (one
 * "iteration" of the LinearSolvers.F90 GSsolver_Mesh* facade, :632-848) */
int pamg_sweep(pamg_handle *h, int level, int n_sweeps);
/* `call restrictor` splitting.F90:10-32 (no-op on the coarsest level) */
int pamg_restrictor(pamg_handle *h, int level);
/* `call get_residual` :725-873 */
int pamg_get_residual(pamg_handle *h, int level);
/* `call prolongator` splitting.F90:38-91 */
int pamg_prolongator(pamg_handle *h, int level);
/* n passes of the n_multigrid loop body :319-379 */
int pamg_vcycle(pamg_handle *h, int n);
/* the time loop :299-381 */
int pamg_run(pamg_handle *h, int ntime, int n_multigrid);
/* launch schedule of pipelined V-cycle calls (fused = 3, halo exchanged once per call).
 * Every operation of a call is local to an un_ele, so tiles need no ordering until the
 * call's end: 1 one launch per cycle; 2 the tiles as two halves on two HIP streams;
 * 3 resident: every cycle of the call in one launch, each tile's state on-chip between
 * cycles; 0 automatic (3 where supported: two levels or more; else one GPU: 1, a partition
 * of a multi-rank run: 2). The state after the call is bitwise the same in all. */
int pamg_set_call_schedule(pamg_handle *h, int schedule);
/* fp64 operations one fused V-cycle of the handle's configuration executes (the resident
 * launch's roofline): its sweeps, residuals, restrictions and prolongation cascades, less each
 * smoother call's last sweep, whose only output (tnew_nonlin) the cycle overwrites unread
 *  */
int pamg_vcycle_flops(pamg_handle *h, double *flops_per_cycle);
int pamg_synchronize(pamg_handle *h);

/* ---- measurement ---- */
/* enable HIP-event timing of the kernel classes in `mask` (bit PAMG_K_*) */
int pamg_timing_enable(pamg_handle *h, unsigned mask);
int pamg_timing_reset(pamg_handle *h);
/* record events around one launch in `every` of each enabled class (the first after a reset,
 * then every `every`-th); timing_read then reports the sampled launches. A HIP event pair
 * between back-to-back launches costs ~10 us; bench.py samples 1 in 10. */
int pamg_timing_stride(pamg_handle *h, int every);
/* launches of class `kid` issued since the reset while its timing was enabled (sampled or not) */
int pamg_timing_issued(pamg_handle *h, int kid, long *issued);
/* total ms, launches and algorithmic HBM bytes of kernel class `kid` since reset */
int pamg_timing_read(pamg_handle *h, int kid, double *ms_total, long *launches, double *bytes_total);
/* the unfused level-1 roofline kernel: `sweeps` launches of one smoother sweep
 * (assembled=0: per-un_ele stencils; assembled=1: per-sub-element 3x3 blocks,
 * block-CSR with one block per block-row, the matrices.F90 format) */
int pamg_sweep_bench(pamg_handle *h, int sweeps, int assembled, double *ms_avg, double *bytes_per_launch);
/* one launch of the same roofline kernel, its output -- one Jacobi sweep of level 1 from
 * tnew_nonlin and RHS (solve_Jacobi :491-497), the state untouched -- copied to host as
 * (3, nsub_1, U): assembled = 0 in the reference's operation order, 1 in the contracted one
 * (arith = 1); the checker of the roofline kernels (tests/test_roofline_kernels.py) */
int pamg_sweep_bench_output(pamg_handle *h, int assembled, double *out);

/* ---- local block solve: replaces FINDInv (matrix_inversion.F90:50-148 = matrices.F90:1618-1716) ----
 * nb n x n matrices, column-major (n, n, nb) host arrays as the reference's
 * `matrix(n,n)`; inverted on the handle's device by the reference's Gauss-Jordan
 * (no pivoting, its zero-pivot row repair and give-up rule), bitwise equal to
 * it. errorflag[q] = 0, or -1 for a matrix the routine calls non-invertible
 * (inverse 0). n <= 8 (element blocks; the reference's dense global inverse of
 * modes 4/8 is out of scope). */
int pamg_block_inverse(pamg_handle *h, int n, long nb, const double *A, double *inv, int *errorflag);
/* tnew = tnew_nonlin = A_e^-1 RHS on `level` (the coarse_solver = 1 step, callable per level) */
int pamg_direct_solve(pamg_handle *h, int level);

/* ---- the matrices.F90 SpMV: replaces csr_mul_array (matrices.F90:172-193) ----
 * The reference's `type sparse` (Structures.F90:196-201): nrows = size(g_iloc) rows (its
 * values are not read), g_jloc 1-based columns and val in storage order; the routine
 * consumes 3 entries per row in that order, so nnz >= 3 nrows. Uploaded once by
 * pamg_csr_create; pamg_csr_mul_array(h, m, n, array(n), result(nrows)) is the call site's
 * `call csr_mul_array(sparse_matrix, array, result)`, bitwise equal to it. */
typedef struct pamg_csr pamg_csr;
int pamg_csr_create(pamg_handle *h, long nrows, long nnz, const int *g_jloc, const double *val, pamg_csr **m);
int pamg_csr_mul_array(pamg_handle *h, pamg_csr *m, long n, const double *array, double *result);
/* the same on device-resident vectors (ordered on the handle's stream, no synchronisation) */
int pamg_csr_mul_array_device(pamg_handle *h, pamg_csr *m, long n, const double *d_array, double *d_result);
int pamg_csr_free(pamg_csr *m);
/* roofline measurement of the csr kernel: average of `reps` launches on device vectors */
int pamg_csr_bench(pamg_handle *h, pamg_csr *m, long n, int reps, double *ms_avg);

/* ---- multi-GPU (one process per GPU, RCCL over xGMI) ---- */
int pamg_comm_unique_id(char out[128]);
/* owner[U] = rank (0-based) owning each un_ele; call before pamg_upload_mesh.
 * nranks == 1 needs no id. The halo (update_overlaps) towards un_eles owned by
 * other ranks is exchanged with grouped ncclSend/ncclRecv after every halo write.
 * RCCL's asynchronous error state is polled at the end of pamg_vcycle / pamg_run and
 * while pamg_synchronize and the getters wait: a failed peer returns PAMG_ERR_COMM (the
 * communicator is aborted) instead of a hang. Every wait for a stream that carries
 * exchanges (pamg_synchronize, the getters, the calls that read state back) is bounded by
 * PAMG_COMM_TIMEOUT_S (seconds, default 120): a rank whose peer stops exchanging returns
 * PAMG_ERR_COMM within that bound. pamg_comm_init itself blocks until every rank has joined
 * (RCCL's bootstrap has no bound, profiles/r06_rccl_init_probe.txt): the launcher bounds it
 * (bench.py: a gloo barrier with a timeout right before it). A failed pamg_comm_init leaves
 * the handle as it was (no communicator, rank or owner map bound). */
int pamg_comm_init(pamg_handle *h, int nranks, int rank, const char id[128], int U, const int *owner);
int pamg_owned_count(pamg_handle *h);
/* one-rank RCCL communicator with a self-peer halo plan: the handle owns the whole mesh, but
 * the halo words across two virtual parts (part[U], any ids) are exchanged exactly as remote
 * words are -- packed into the send buffer, grouped ncclSend / ncclRecv to this rank itself,
 * unpacked -- so the RCCL transport (exchange(), the async error poll) runs on one GPU. The
 * state is bitwise that of the plain single domain (tests/test_rccl_self.py). Call before
 * pamg_upload_mesh. */
int pamg_comm_init_self(pamg_handle *h, const char id[128], int U, const int *part);
/* single-process exchange of the packed halo of `level` between n partition
 * handles (created with pamg_comm_init(id = NULL)): the same send/recv
 * segments RCCL would carry, copied device to device, then unpacked */
int pamg_halo_loopback(pamg_handle *const *hs, int n, int level);
/* single-process device-copy transport: binds the n detached partition handles of one owner
 * map (ranks 0..n-1, pamg_comm_init(id = NULL), meshes uploaded) into a group whose halo
 * exchange runs the RCCL path itself -- halo_async on the comm stream, the double-buffered send
 * words, join_comm -- with ncclSend / ncclRecv replaced by device-to-device copies between the
 * handles. Each handle must then be driven by its own host thread (ranks meet at every
 * exchange, as grouped send / recv calls do); a rank waiting longer than PAMG_COMM_TIMEOUT_S
 * (default 120 s) for a peer returns PAMG_ERR_COMM. */
int pamg_comm_local_group(pamg_handle *const *hs, int n);
/* RCCL version (ncclGetVersion) and the path of the librccl this library is bound to;
 * returns 0 (no communicator), 1 (RCCL) or 2 (local group), < 0 on error */
int pamg_comm_info(pamg_handle *h, int *version, char *lib_path, int len);
/* the last pamg_vcycle call whose per-call exchange started early (timing class PAMG_K_HALO_EARLY enabled):
 * t[0] the exchange's start (the comm stream past the device signal), t[1] its end, t[2] the end of the
 * resident launch -- microseconds from the launch's start (t[1] < t[2]: the exchange was hidden). PAMG_ERR_STATE
 * if no such call was recorded since the timing was enabled */
int pamg_early_exchange_times(pamg_handle *h, double t[3]);

/* ---- host-only halo plan (tooling / CPU tests of the partitioned exchange) ---- */
typedef struct pamg_plan pamg_plan;
int pamg_plan_build(int U, const double *X, const int *neig, const int *fneig, const int *dir, int n_split,
                    int level, int nranks, int rank, const int *owner, pamg_plan **out);
/* sizes[6] = n_owned, n_local, n_bc, n_remote, n_recv, n_peers */
int pamg_plan_sizes(const pamg_plan *p, int *sizes);
/* any pointer may be NULL; bc_dst / bc_val hold (a, b) pairs; offsets have n_peers + 1 entries */
int pamg_plan_get(const pamg_plan *p, int *owned, int *local_src, int *local_dst, int *bc_dst, double *bc_val,
                  int *remote_src, int *peers, int *send_off, int *recv_dst, int *recv_off);
void pamg_plan_free(pamg_plan *p);

int pamg_last_error(pamg_handle *h, char *buf, int len);
int pamg_destroy(pamg_handle *h);

#ifdef __cplusplus
}
#endif
#endif /* PAMG_H */
