"""pamg -- MI355X-native multigrid hot path of Amin-Nadimy/P-A_multigrids.

Python host mirror over libpamg.so (HIP kernels for gfx950 behind the C-ABI in
include/pamg.h). See DESIGN.md.
"""
from ._lib import (K_NAMES, RESIDUAL, RHS, SOURCE, TNEW, TNEW_NONLIN, TOLD, PamgError, lib)  # noqa: F401
from .solver import Mesh, SemiImplicitIterative, Sparse, csr_mul_array, default_params, unique_id  # noqa: F401

__all__ = ["Mesh", "SemiImplicitIterative", "default_params", "unique_id", "lib", "PamgError",
           "TNEW", "TOLD", "RHS", "RESIDUAL", "TNEW_NONLIN", "SOURCE", "K_NAMES"]
