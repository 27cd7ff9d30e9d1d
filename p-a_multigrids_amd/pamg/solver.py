"""Python host mirror of the reference's mode-9 driver over libpamg.

`Mesh` replaces ReadMSH (Msh2Tri.F90:132-334); `SemiImplicitIterative` owns a
libpamg handle and exposes one method per reference call site, named after the
reference subroutines (transport_tri_semi.F90:299-381, splitting.F90:10-91):
smoother, restrictor, get_residual, prolongator, plus the driver loop. Field
arrays use the reference's Fortran shape (3, nsub, U), fp64.
"""
import ctypes as C
import os

import numpy as np

from ._lib import (PAMG_OK, PamgError, PamgParams, TNEW, TOLD, RHS, RESIDUAL, TNEW_NONLIN, K_NAMES, lib)


def _check(fn, rc, h=None):
    if rc != PAMG_OK:
        msg = ""
        if h:
            buf = C.create_string_buffer(512)
            lib().pamg_last_error(h, buf, 512)
            msg = buf.value.decode(errors="replace")
        raise PamgError(fn, rc, msg)


class Mesh:
    """Unstructured triangle mesh + reference topology (Mesh%X/Neig/fNeig/Dir/region_id)."""

    def __init__(self, ptr):
        L = lib()
        self._ptr = ptr
        U = C.c_int()
        _check("pamg_msh_size", L.pamg_msh_size(ptr, C.byref(U)))
        self.U = U.value
        self.X = np.zeros(6 * self.U, np.float64)
        self.region = np.zeros(self.U, np.int32)
        self.neig = np.zeros(3 * self.U, np.int32)
        self.fneig = np.zeros(3 * self.U, np.int32)
        self.dir = np.zeros(3 * self.U, np.int32)
        _check("pamg_msh_get", L.pamg_msh_get(ptr, self.X, self.region, self.neig, self.fneig, self.dir))

    @classmethod
    def read(cls, path):
        p = C.c_void_p()
        _check("pamg_msh_read", lib().pamg_msh_read(str(path).encode(), C.byref(p)))
        return cls(p)

    @classmethod
    def strip(cls, nx, ny, lx=1.0, ly=1.0 / 15.0):
        p = C.c_void_p()
        _check("pamg_msh_strip", lib().pamg_msh_strip(nx, ny, lx, ly, C.byref(p)))
        return cls(p)

    @classmethod
    def load(cls, path):
        """binary mesh cache written by save() (pamg_msh_load)"""
        p = C.c_void_p()
        _check("pamg_msh_load", lib().pamg_msh_load(os.fsencode(path), C.byref(p)))
        return cls(p)

    @classmethod
    def read_cached(cls, msh_path, cache_path):
        """ReadMSH with a binary cache: (mesh, hit) -- the .msh is parsed only when the cache is
        missing or was made from other file contents (pamg_msh_read_cached)"""
        p, hit = C.c_void_p(), C.c_int()
        _check("pamg_msh_read_cached", lib().pamg_msh_read_cached(os.fsencode(msh_path), os.fsencode(cache_path),
                                                                  C.byref(p), C.byref(hit)))
        return cls(p), bool(hit.value)

    def save(self, path):
        _check("pamg_msh_save", lib().pamg_msh_save(self._ptr, os.fsencode(path)))

    def write_msh(self, path):
        """gmsh 2.2 ASCII (pamg_msh_write), readable by the reference's ReadMSH"""
        _check("pamg_msh_write", lib().pamg_msh_write(self._ptr, os.fsencode(path)))

    def __del__(self):
        if getattr(self, "_ptr", None):
            lib().pamg_msh_free(self._ptr)
            self._ptr = None

    def x_strip_owner(self, nranks):
        """Contiguous partition by element centroid x (balanced strips), 0-based ranks."""
        cx = self.X.reshape(self.U, 6)[:, 0::2].mean(axis=1)
        order = np.argsort(cx, kind="stable")
        owner = np.empty(self.U, np.int32)
        for r, chunk in enumerate(np.array_split(order, nranks)):
            owner[chunk] = r
        return owner

    def block_owner(self, nranks):
        """Generic.F90:387-401 getProcessor: contiguous blocks of un_ele index."""
        owner = np.empty(self.U, np.int32)
        for r, chunk in enumerate(np.array_split(np.arange(self.U), nranks)):
            owner[chunk] = r
        return owner


def default_params(**kw):
    p = PamgParams()
    lib().pamg_default_params(C.byref(p))
    for k, v in kw.items():
        if not hasattr(p, k):
            raise TypeError(f"unknown parameter {k}")
        setattr(p, k, v)
    return p


class SemiImplicitIterative:
    """Device-resident multigrid state for one mesh (one GPU / rank)."""

    def __init__(self, mesh, n_split, multi_levels, n_smooth=4, solver=3, n_coarse=15, device=0,
                 dt=1.0 * 0.0000125, k=1.0, omega=0.8, halo_mode=0, comm=None, fused=3, coarse_solver=0,
                 arith=0, halo_exchange=0, cycle=0, op=0, self_peer=None):
        self.L = lib()
        self.mesh = mesh
        self.params = default_params(n_split=n_split, multi_levels=multi_levels, n_smooth=n_smooth,
                                     solver=solver, n_coarse=n_coarse, device=device, dt=dt, k=k,
                                     omega=omega, halo_mode=halo_mode, fused=fused, coarse_solver=coarse_solver,
                                     arith=arith, halo_exchange=halo_exchange, cycle=cycle, op=op)
        h = C.c_void_p()
        _check("pamg_create", self.L.pamg_create(C.byref(self.params), C.byref(h)))
        self.h = h
        if comm is not None:
            nranks, rank, uid, owner = comm
            owner = np.ascontiguousarray(owner, np.int32)
            self._call("pamg_comm_init", nranks, rank, uid, mesh.U, owner)
        if self_peer is not None:
            # one-rank RCCL communicator whose halo plan sends the words across the parts of
            # self_peer = (unique id, part[U]) to this rank itself (pamg_comm_init_self)
            uid, part = self_peer
            self._call("pamg_comm_init_self", uid, mesh.U, np.ascontiguousarray(part, np.int32))
        self._call("pamg_upload_mesh", mesh.U, mesh.X, mesh.region, mesh.neig, mesh.fneig, mesh.dir)
        self.U = self.L.pamg_owned_count(self.h)
        self.n_split, self.levels = n_split, multi_levels

    def _call(self, name, *args):
        rc = getattr(self.L, name)(self.h, *args)
        _check(name, rc, self.h)
        return rc

    def close(self):
        if getattr(self, "h", None):
            self.L.pamg_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()

    # ---- state -----------------------------------------------------------
    def nsub(self, level):
        return 4 ** (self.n_split - level + 1)

    def get(self, what, level=1):
        if what == TNEW_NONLIN:
            level = self.L.pamg_tnn_level(self.h)
        out = np.empty(3 * self.nsub(level) * self.U, np.float64)
        self._call("pamg_get_state", level, what, out)
        return out.reshape((3, self.nsub(level), self.U), order="F")

    def set(self, what, level, arr):
        a = np.ascontiguousarray(np.asarray(arr, np.float64).reshape(-1, order="F"))
        assert a.size == 3 * self.nsub(level) * self.U
        self._call("pamg_set_state", level, what, a)

    def overlap(self):
        n = (2 ** self.n_split) * 3 * 3 * self.U
        a, b = np.empty(n), np.empty(n)
        self._call("pamg_get_overlap", a, b)
        shp = ((2 ** self.n_split) * 3, 3, self.U)
        return a.reshape(shp, order="F"), b.reshape(shp, order="F")

    def state(self):
        d = {}
        for l in range(1, self.levels + 1):
            d[f"tnew_L{l}"] = self.get(TNEW, l)
            d[f"told_L{l}"] = self.get(TOLD, l)
            d[f"RHS_L{l}"] = self.get(RHS, l)
            d[f"res_L{l}"] = self.get(RESIDUAL, l)
        d["tnew_nonlin"] = self.get(TNEW_NONLIN)
        return d

    # ---- the hot path (one method per reference call site) ---------------
    def begin_timestep(self): self._call("pamg_begin_timestep")
    def copy_to_tnn(self, level): self._call("pamg_copy_to_nonlin", level)
    def smoother(self, level, n_calls=1): self._call("pamg_smoother", level, n_calls)
    def restrictor(self, level): self._call("pamg_restrictor", level)
    def get_residual(self, level): self._call("pamg_get_residual", level)
    def prolongator(self, level): self._call("pamg_prolongator", level)
    def vcycle(self, n=1): self._call("pamg_vcycle", n)
    def direct_solve(self, level): self._call("pamg_direct_solve", level)

    def write_vtu(self, path, ascii=False):
        """get_vtu (get_vtk_files.F90:10-165) of the level-1 solution at full precision."""
        self._call("pamg_write_vtu", os.fsencode(path), 1 if ascii else 0)

    def block_inverse(self, A):
        """FINDInv (matrix_inversion.F90:50-148) of a batch A (n, n, nb), column-major as the
        reference's matrix(n, n); returns (inverses (n, n, nb), errorflags (nb,))."""
        A = np.asarray(A, np.float64)
        n, nb = A.shape[0], A.shape[2]
        a = np.ascontiguousarray(A.reshape(-1, order="F"))
        inv = np.empty_like(a)
        err = np.empty(nb, np.int32)
        self._call("pamg_block_inverse", n, nb, a, inv, err)
        return inv.reshape((n, n, nb), order="F"), err
    def run(self, ntime=2, n_multigrid=2): self._call("pamg_run", ntime, n_multigrid)

    def comm_info(self):
        """(transport, RCCL version, path of the librccl libpamg is bound to); transport is
        "none", "rccl" or "local" (pamg_comm_local_group)"""
        v = C.c_int()
        buf = C.create_string_buffer(1024)
        rc = self.L.pamg_comm_info(self.h, C.byref(v), buf, 1024)
        if rc < 0:
            _check("pamg_comm_info", rc, self.h)
        return {0: "none", 1: "rccl", 2: "local"}[rc], v.value, buf.value.decode(errors="replace")
    def synchronize(self): self._call("pamg_synchronize")

    def early_exchange_times(self):
        """the last call whose per-call exchange started early (timing class halo_early enabled):
        (exchange start, exchange end, launch end) in us from the launch's start, or None"""
        t = np.zeros(3)
        rc = self.L.pamg_early_exchange_times(self.h, t)
        if rc == -4:   # PAMG_ERR_STATE: none recorded
            return None
        if rc < 0:
            _check("pamg_early_exchange_times", rc, self.h)
        return tuple(float(v) for v in t)

    # ---- measurement ------------------------------------------------------
    def timing_enable(self, mask): self._call("pamg_timing_enable", mask)
    def timing_reset(self): self._call("pamg_timing_reset")
    def timing_stride(self, every): self._call("pamg_timing_stride", every)

    def vcycle_flops(self):
        """fp64 operations of one V-cycle (pamg_vcycle_flops)"""
        f = C.c_double()
        self._call("pamg_vcycle_flops", C.byref(f))
        return f.value

    def set_call_schedule(self, schedule):
        """Pipelined calls: 0 automatic, 1 one launch per cycle, 2 two tile streams, 3 resident
        (pamg_set_call_schedule)."""
        self._call("pamg_set_call_schedule", schedule)

    def timing(self):
        out = {}
        for kid, name in enumerate(K_NAMES):
            ms, n, by = C.c_double(), C.c_long(), C.c_double()
            self._call("pamg_timing_read", kid, C.byref(ms), C.byref(n), C.byref(by))
            iss = C.c_long()
            self._call("pamg_timing_issued", kid, C.byref(iss))
            out[name] = dict(ms=ms.value, launches=n.value, bytes=by.value, issued=iss.value)
        return out

    def sweep_bench(self, sweeps, assembled):
        ms, by = C.c_double(), C.c_double()
        self._call("pamg_sweep_bench", sweeps, 1 if assembled else 0, C.byref(ms), C.byref(by))
        return ms.value, by.value

    def sweep_bench_output(self, assembled):
        """one launch of the level-1 roofline sweep kernel (assembled: the block-CSR operator in the
        contracted arithmetic; else the per-un_ele stencil in the reference's order) from tnew_nonlin
        and RHS; its output as (3, nsub_1, U) (pamg_sweep_bench_output)"""
        out = np.empty(3 * self.nsub(1) * self.U, np.float64)
        self._call("pamg_sweep_bench_output", 1 if assembled else 0, out)
        return out.reshape((3, self.nsub(1), self.U), order="F")


class Sparse:
    """The reference's `type sparse` (Structures.F90:196-201) resident on a handle's device:
    csr_mul_array (matrices.F90:172-193) as .mul_array(array) -> result(nrows)."""

    def __init__(self, solver, g_iloc, g_jloc, val):
        self.s = solver
        self.nrows = int(np.asarray(g_iloc).size)
        j = np.ascontiguousarray(g_jloc, np.int32)
        v = np.ascontiguousarray(val, np.float64)
        m = C.c_void_p()
        solver._call("pamg_csr_create", self.nrows, j.size, j, v, C.byref(m))
        self.m = m

    def mul_array(self, array):
        a = np.ascontiguousarray(array, np.float64)
        out = np.empty(self.nrows)
        self.s._call("pamg_csr_mul_array", self.m, a.size, a, out)
        return out

    def mul_array_device(self, n, d_array, d_result):
        """device pointers (e.g. torch tensors' data_ptr()), ordered on the handle's stream"""
        self.s._call("pamg_csr_mul_array_device", self.m, n, C.c_void_p(d_array), C.c_void_p(d_result))

    def bench(self, n, reps=20):
        """average ms per launch of the device kernel (HIP events)"""
        ms = C.c_double()
        self.s._call("pamg_csr_bench", self.m, n, reps, C.byref(ms))
        return ms.value

    def close(self):
        if getattr(self, "m", None):
            self.s.L.pamg_csr_free(self.m)
            self.m = None

    def __del__(self):
        self.close()


def csr_mul_array(solver, sparse_matrix, array):
    """matrices.F90:172 `call csr_mul_array(sparse_matrix, array, result)`; sparse_matrix is
    (g_iloc, g_jloc, val) or a Sparse."""
    if not isinstance(sparse_matrix, Sparse):
        sparse_matrix = Sparse(solver, *sparse_matrix)
    return sparse_matrix.mul_array(array)


def unique_id():
    buf = C.create_string_buffer(128)
    _check("pamg_comm_unique_id", lib().pamg_comm_unique_id(buf))
    return buf.raw


def halo_loopback(solvers, level=1):
    """Exchange the packed halo between partition handles of one process (no RCCL)."""
    arr = (C.c_void_p * len(solvers))(*[s.h for s in solvers])
    _check("pamg_halo_loopback", lib().pamg_halo_loopback(arr, len(solvers), level))


def local_group(solvers):
    """Bind detached partition handles (ranks 0..n-1 of one owner map) into one process's
    device-copy transport (pamg_comm_local_group): their exchanges then run the RCCL path
    with device copies in place of ncclSend/ncclRecv. Drive them with run_ranks."""
    arr = (C.c_void_p * len(solvers))(*[s.h for s in solvers])
    rc = lib().pamg_comm_local_group(arr, len(solvers))
    if rc != PAMG_OK:
        _check("pamg_comm_local_group", rc, solvers[0].h)


def run_ranks(solvers, fn):
    """fn(solver) on every partition, one host thread per rank (the ranks of a local group meet
    at every halo exchange); re-raises the first error."""
    import threading
    errs = [None] * len(solvers)

    def body(i):
        try:
            fn(solvers[i])
        except BaseException as e:  # noqa: BLE001 -- reported to the caller
            errs[i] = e

    ts = [threading.Thread(target=body, args=(i,)) for i in range(len(solvers))]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    for e in errs:
        if e is not None:
            raise e


class HaloPlan:
    """Host-only halo plan of update_overlaps for one rank of a partitioned mesh."""

    def __init__(self, mesh, n_split, level, nranks, rank, owner):
        L = lib()
        owner = np.ascontiguousarray(owner if owner is not None else np.zeros(mesh.U), np.int32)
        p = C.c_void_p()
        _check("pamg_plan_build", L.pamg_plan_build(mesh.U, mesh.X, mesh.neig, mesh.fneig, mesh.dir, n_split,
                                                    level, nranks, rank, owner, C.byref(p)))
        s = np.zeros(6, np.int32)
        L.pamg_plan_sizes(p, s)
        n_owned, n_local, n_bc, n_remote, n_recv, n_peers = (int(v) for v in s)
        self.owned = np.zeros(n_owned, np.int32)
        self.local_src, self.local_dst = np.zeros(n_local, np.int32), np.zeros(n_local, np.int32)
        self.bc_dst, self.bc_val = np.zeros(2 * n_bc, np.int32), np.zeros(2 * n_bc, np.float64)
        self.remote_src = np.zeros(n_remote, np.int32)
        self.peers = np.zeros(n_peers, np.int32)
        self.send_off = np.zeros(n_peers + 1, np.int32)
        self.recv_dst = np.zeros(n_recv, np.int32)
        self.recv_off = np.zeros(n_peers + 1, np.int32)
        ptr = lambda a: a.ctypes.data if a.size else None  # noqa: E731
        _check("pamg_plan_get", L.pamg_plan_get(
            p, ptr(self.owned), ptr(self.local_src), ptr(self.local_dst), ptr(self.bc_dst), ptr(self.bc_val),
            ptr(self.remote_src), ptr(self.peers), self.send_off.ctypes.data, ptr(self.recv_dst),
            self.recv_off.ctypes.data))
        L.pamg_plan_free(p)
