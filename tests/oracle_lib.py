"""ctypes binding of the C oracle (oracle/pamg_oracle.c -> oracle/_build/liborc.so).

TEST INFRASTRUCTURE: only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg use this module, and only as the checker / CPU baseline.
Field arrays are returned in the reference's Fortran shape (3, nsub, U).
"""
import ctypes as C
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
# ORACLE_LIB: another build of the same checker (the host sanitizer build, scripts/asan_cpu_tests.sh)
LIB_PATH = os.environ.get("ORACLE_LIB") or os.path.join(ORACLE_DIR, "_build", "liborc.so")

TNEW, TOLD, RHS, RES, TNN, SOURCE = 0, 1, 2, 3, 4, 5


class OrcCfg(C.Structure):
    _fields_ = [("n_split", C.c_int), ("levels", C.c_int), ("n_smooth", C.c_int),
                ("n_coarse", C.c_int), ("solver", C.c_int), ("ntime", C.c_int),
                ("n_multigrid", C.c_int), ("dt", C.c_double), ("k", C.c_double),
                ("omega", C.c_double), ("theta", C.c_double), ("coarse_solver", C.c_int), ("op", C.c_int),
                ("arith", C.c_int)]


_lib = None


def build():
    subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        P = C.c_void_p
        dp = np.ctypeslib.ndpointer(np.float64, flags="C_CONTIGUOUS")
        ip = np.ctypeslib.ndpointer(np.int32, flags="C_CONTIGUOUS")
        L.orc_msh_count.argtypes = [C.c_char_p]
        L.orc_msh_load.argtypes = [C.c_char_p, C.c_int, dp, ip, ip, ip, ip]
        L.orc_create.restype = P
        L.orc_create.argtypes = [C.POINTER(OrcCfg), C.c_int, dp, ip, ip, ip, ip]
        L.orc_free.argtypes = [P]
        L.orc_get.restype = C.c_long
        L.orc_get.argtypes = [P, C.c_int, C.c_int, C.c_void_p]
        L.orc_set.argtypes = [P, C.c_int, C.c_int, dp]
        L.orc_set_source.argtypes = [P, C.c_void_p]
        L.orc_tnn_level.argtypes = [P]
        L.orc_get_overlap.argtypes = [P, dp, dp]
        L.orc_level_geometry.argtypes = [P, C.c_int, dp, dp, dp, dp]
        dpc = np.ctypeslib.ndpointer(np.float64, flags="C_CONTIGUOUS")
        L.orc_findinv.restype = C.c_int
        L.orc_findinv.argtypes = [C.c_int, dpc, dpc]
        ipc = np.ctypeslib.ndpointer(np.int32, flags="C_CONTIGUOUS")
        L.orc_csr_mul_array.restype = None
        L.orc_csr_mul_array.argtypes = [C.c_long, ipc, dpc, dpc, dpc]
        L.orc_sweep_once.restype = None
        L.orc_sweep_once.argtypes = [P, C.c_int, C.c_int, dpc, dpc, dpc]
        for name in ("orc_copy_to_tnn", "orc_smoother", "orc_get_residual", "orc_restrictor",
                     "orc_prolongator", "orc_update_overlaps", "orc_direct_solve"):
            getattr(L, name).argtypes = [P, C.c_int]
        for name in ("orc_begin_timestep", "orc_vcycle", "orc_run", "orc_vcycle_corrected"):
            getattr(L, name).argtypes = [P]
        _lib = L
    return _lib


class Mesh:
    """Reference topology: X (2,3,U), region (U), Neig/fNeig/Dir (3,U), 1-based neighbours."""

    def __init__(self, U, X, region, neig, fneig, dir_):
        self.U, self.X, self.region, self.neig, self.fneig, self.dir = U, X, region, neig, fneig, dir_


def read_msh(path):
    L = lib()
    U = L.orc_msh_count(path.encode())
    if U < 0:
        raise IOError(f"oracle could not read {path} ({U})")
    X = np.zeros(6 * U, np.float64)
    reg = np.zeros(U, np.int32)
    ne, fn, di = (np.zeros(3 * U, np.int32) for _ in range(3))
    rc = L.orc_msh_load(path.encode(), U, X, reg, ne, fn, di)
    if rc != 0:
        raise IOError(f"oracle msh load failed {rc}")
    return Mesh(U, X, reg, ne, fn, di)


class Oracle:
    def __init__(self, mesh, n_split, levels, n_smooth=4, solver=3, ntime=2, n_multigrid=2,
                 n_coarse=15, dt=1.25e-5, k=1.0, omega=0.8, theta=1.0, coarse_solver=0, arith=0, op=0):
        self.L = lib()
        self.mesh = mesh
        self.cfg = OrcCfg(n_split, levels, n_smooth, n_coarse, solver, ntime, n_multigrid, dt, k, omega, theta,
                          coarse_solver, op, arith)
        self.h = self.L.orc_create(C.byref(self.cfg), mesh.U, mesh.X, mesh.region, mesh.neig,
                                   mesh.fneig, mesh.dir)
        if not self.h:
            raise ValueError("orc_create rejected the configuration")
        self.n_split, self.levels = n_split, levels

    def __del__(self):
        if getattr(self, "h", None):
            self.L.orc_free(self.h)
            self.h = None

    def nsub(self, level):
        return 4 ** (self.n_split - level + 1)

    def get(self, what, level=1):
        n = self.L.orc_get(self.h, what, level, None)
        out = np.empty(n, np.float64)
        self.L.orc_get(self.h, what, level, out.ctypes.data)
        lv = self.L.orc_tnn_level(self.h) if what == TNN else level
        return out.reshape((3, self.nsub(lv), self.mesh.U), order="F")

    def set(self, what, level, arr):
        a = np.ascontiguousarray(np.asarray(arr, np.float64).reshape(-1, order="F"))
        assert self.L.orc_set(self.h, what, level, a) == 0

    def set_source(self, src1):
        """test hook: level 1's cascaded source term s' (3, nsub_1, U) used instead of evaluating
        it with the host's sin (None: evaluate it again)"""
        if src1 is None:
            assert self.L.orc_set_source(self.h, None) == 0
            return
        a = np.ascontiguousarray(np.asarray(src1, np.float64).reshape(-1, order="F"))
        assert a.size == 3 * self.nsub(1) * self.mesh.U
        self._src = a
        assert self.L.orc_set_source(self.h, a.ctypes.data) == 0

    def overlap(self):
        n = (2 ** self.n_split) * 3 * 3 * self.mesh.U
        a, b = np.empty(n), np.empty(n)
        self.L.orc_get_overlap(self.h, a, b)
        shp = ((2 ** self.n_split) * 3, 3, self.mesh.U)
        return a.reshape(shp, order="F"), b.reshape(shp, order="F")

    def geometry(self, level):
        U = self.mesh.U
        dw, M, Kd, ml = np.empty(3 * U), np.empty(9 * U), np.empty(9 * U), np.empty(3 * U)
        self.L.orc_level_geometry(self.h, level, dw, M, Kd, ml)
        return (dw.reshape((3, U), order="F"), M.reshape((3, 3, U), order="F"),
                Kd.reshape((3, 3, U), order="F"), ml.reshape((3, U), order="F"))

    def copy_to_tnn(self, l): self.L.orc_copy_to_tnn(self.h, l)
    def smoother(self, l): self.L.orc_smoother(self.h, l)
    def get_residual(self, l): self.L.orc_get_residual(self.h, l)
    def restrictor(self, l): self.L.orc_restrictor(self.h, l)
    def prolongator(self, l): self.L.orc_prolongator(self.h, l)
    def update_overlaps(self, l): self.L.orc_update_overlaps(self.h, l)
    def direct_solve(self, l): self.L.orc_direct_solve(self.h, l)
    def begin_timestep(self): self.L.orc_begin_timestep(self.h)
    def vcycle(self): self.L.orc_vcycle(self.h)
    def vcycle_corrected(self): self.L.orc_vcycle_corrected(self.h)
    def run(self): self.L.orc_run(self.h)

    def sweep_once(self, level, arith, x, b):
        """one Jacobi sweep of `level` from x and b, (3, nsub, U) each, the state untouched
        (orc_sweep_once: the reference's operation order, or the contracted one with arith = 1)"""
        xf = np.ascontiguousarray(np.asarray(x, np.float64).reshape(-1, order="F"))
        bf = np.ascontiguousarray(np.asarray(b, np.float64).reshape(-1, order="F"))
        out = np.empty_like(xf)
        self.L.orc_sweep_once(self.h, level, arith, xf, bf, out)
        return out.reshape((3, self.nsub(level), self.mesh.U), order="F")

    def state(self):
        d = {}
        for l in range(1, self.levels + 1):
            d[f"tnew_L{l}"] = self.get(TNEW, l)
            d[f"told_L{l}"] = self.get(TOLD, l)
            d[f"RHS_L{l}"] = self.get(RHS, l)
            d[f"res_L{l}"] = self.get(RES, l)
        d["tnew_nonlin"] = self.get(TNN)
        return d


def csr_mul_array(nrows, jloc, val, array):
    """csr_mul_array restatement (oracle/pamg_oracle.c orc_csr_mul_array)."""
    out = np.empty(nrows)
    lib().orc_csr_mul_array(nrows, np.ascontiguousarray(jloc, np.int32), np.ascontiguousarray(val, np.float64),
                            np.ascontiguousarray(array, np.float64), out)
    return out


def findinv(A):
    """FINDInv restatement (oracle/pamg_oracle.c orc_findinv) of a batch A (n, n, nb)."""
    A = np.asarray(A, np.float64)
    n, nb = A.shape[0], A.shape[2]
    inv = np.empty_like(A)
    err = np.empty(nb, np.int32)
    for q in range(nb):
        o = np.empty(n * n)
        err[q] = lib().orc_findinv(n, np.ascontiguousarray(A[:, :, q].reshape(-1, order="F")), o)
        inv[:, :, q] = o.reshape((n, n), order="F")
    return inv, err
