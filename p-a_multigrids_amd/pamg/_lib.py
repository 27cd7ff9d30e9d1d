"""ctypes loader for the in-tree libpamg.so (include/pamg.h).

The library is the product: there is no Python / CPU fallback. If libpamg.so
is missing the import fails loudly; build it with `make -C p-a_multigrids_amd`
or `python -c "import __graft_entry__ as g; g.build()"`.
"""
import ctypes as C
import os

import numpy as np

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
# PAMG_LIB: an alternative in-tree build of the same library (A/B timing of kernel variants)
LIB_PATH = os.environ.get("PAMG_LIB") or os.path.join(PKG_DIR, "libpamg.so")

PAMG_OK = 0
ERRORS = {-1: "PAMG_ERR_ARG", -2: "PAMG_ERR_HIP", -3: "PAMG_ERR_IO", -4: "PAMG_ERR_STATE",
          -5: "PAMG_ERR_COMM", -6: "PAMG_ERR_NODEV"}

TNEW, TOLD, RHS, RESIDUAL, TNEW_NONLIN, SOURCE = 0, 1, 2, 3, 4, 5
(K_SMOOTH_L1, K_SMOOTH, K_RESIDUAL, K_RESTRICT, K_PROLONG, K_RHS, K_HALO, K_SWEEP_BENCH, K_VCYCLE,
 K_VCYCLE_COARSE) = range(10)
K_NAMES = ["smooth_L1", "smooth", "residual", "restrict", "prolong", "rhs", "halo", "sweep_bench", "vcycle",
           "vcycle_coarse", "vcycle_pipe", "vcycle_rhsf", "vcycle_res", "vcycle_res_rhsf", "vcycle_corr",
           "halo_early", "face_fallback", "coarse_gather"]


class PamgParams(C.Structure):
    _fields_ = [("n_split", C.c_int), ("multi_levels", C.c_int), ("n_smooth", C.c_int),
                ("n_coarse", C.c_int), ("solver", C.c_int), ("device", C.c_int),
                ("dt", C.c_double), ("k", C.c_double), ("omega", C.c_double), ("theta", C.c_double),
                ("halo_mode", C.c_int), ("fused", C.c_int), ("coarse_solver", C.c_int), ("arith", C.c_int),
                ("halo_exchange", C.c_int), ("cycle", C.c_int), ("op", C.c_int), ("reserved", C.c_int * 1)]


class PamgError(RuntimeError):
    def __init__(self, fn, rc, msg=""):
        super().__init__(f"{fn} failed: {ERRORS.get(rc, rc)} {msg}".strip())
        self.rc = rc


_lib = None


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"libpamg.so not built at {LIB_PATH} (run make -C p-a_multigrids_amd)")
    L = C.CDLL(LIB_PATH)
    P, I, D = C.c_void_p, C.c_int, C.c_double
    dp = np.ctypeslib.ndpointer(np.float64, flags="C_CONTIGUOUS")
    ip = np.ctypeslib.ndpointer(np.int32, flags="C_CONTIGUOUS")
    sig = {
        "pamg_version": (I, []),
        "pamg_default_params": (None, [C.POINTER(PamgParams)]),
        "pamg_msh_read": (I, [C.c_char_p, C.POINTER(P)]),
        "pamg_msh_strip": (I, [I, I, D, D, C.POINTER(P)]),
        "pamg_msh_write": (I, [P, C.c_char_p]),
        "pamg_msh_save": (I, [P, C.c_char_p]),
        "pamg_msh_load": (I, [C.c_char_p, C.POINTER(P)]),
        "pamg_msh_read_cached": (I, [C.c_char_p, C.c_char_p, C.POINTER(P), C.POINTER(I)]),
        "pamg_msh_size": (I, [P, C.POINTER(I)]),
        "pamg_msh_get": (I, [P, dp, ip, ip, ip, ip]),
        "pamg_msh_free": (None, [P]),
        "pamg_create": (I, [C.POINTER(PamgParams), C.POINTER(P)]),
        "pamg_upload_mesh": (I, [P, I, dp, ip, ip, ip, ip]),
        "pamg_nsub": (I, [P, I]),
        "pamg_set_state": (I, [P, I, I, dp]),
        "pamg_get_state": (I, [P, I, I, dp]),
        "pamg_get_overlap": (I, [P, dp, dp]),
        "pamg_tnn_level": (I, [P]),
        "pamg_begin_timestep": (I, [P]),
        "pamg_copy_to_nonlin": (I, [P, I]),
        "pamg_smoother": (I, [P, I, I]),
        "pamg_sweep": (I, [P, I, I]),
        "pamg_restrictor": (I, [P, I]),
        "pamg_get_residual": (I, [P, I]),
        "pamg_prolongator": (I, [P, I]),
        "pamg_vcycle": (I, [P, I]),
        "pamg_run": (I, [P, I, I]),
        "pamg_synchronize": (I, [P]),
        "pamg_timing_enable": (I, [P, C.c_uint]),
        "pamg_timing_reset": (I, [P]),
        "pamg_timing_stride": (I, [P, I]),
        "pamg_set_call_schedule": (I, [P, I]),
        "pamg_vcycle_flops": (I, [P, C.POINTER(C.c_double)]),
        "pamg_timing_issued": (I, [P, I, C.POINTER(C.c_long)]),
        "pamg_timing_read": (I, [P, I, C.POINTER(D), C.POINTER(C.c_long), C.POINTER(D)]),
        "pamg_sweep_bench": (I, [P, I, I, C.POINTER(D), C.POINTER(D)]),
        "pamg_sweep_bench_output": (I, [P, I, dp]),
        "pamg_block_inverse": (I, [P, I, C.c_long, dp, dp, ip]),
        "pamg_direct_solve": (I, [P, I]),
        "pamg_write_vtu": (I, [P, C.c_char_p, I]),
        "pamg_csr_create": (I, [P, C.c_long, C.c_long, ip, dp, C.POINTER(P)]),
        "pamg_csr_mul_array": (I, [P, P, C.c_long, dp, dp]),
        "pamg_csr_mul_array_device": (I, [P, P, C.c_long, C.c_void_p, C.c_void_p]),
        "pamg_csr_free": (I, [P]),
        "pamg_csr_bench": (I, [P, P, C.c_long, I, C.POINTER(D)]),
        "pamg_comm_unique_id": (I, [C.c_char_p]),
        "pamg_comm_init": (I, [P, I, I, C.c_char_p, I, ip]),
        "pamg_owned_count": (I, [P]),
        "pamg_halo_loopback": (I, [C.POINTER(P), I, I]),
        "pamg_comm_local_group": (I, [C.POINTER(P), I]),
        "pamg_comm_init_self": (I, [P, C.c_char_p, I, ip]),
        "pamg_comm_info": (I, [P, C.POINTER(I), C.c_char_p, I]),
        "pamg_early_exchange_times": (I, [P, dp]),
        "pamg_plan_build": (I, [I, dp, ip, ip, ip, I, I, I, I, ip, C.POINTER(P)]),
        "pamg_plan_sizes": (I, [P, ip]),
        "pamg_plan_get": (I, [P] + [C.c_void_p] * 10),
        "pamg_plan_free": (None, [P]),
        "pamg_last_error": (I, [P, C.c_char_p, I]),
        "pamg_destroy": (I, [P]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L
