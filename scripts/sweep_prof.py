"""The level-1 roofline kernels on their own (for rocprofv3 kernel stats and PMC passes):
k_sweep_stencil and k_sweep_assembled on untitled8192 at n_split = 5 (8,388,608 sub-elements),
and k_csr_mul_array over the same operator size (25.2 M rows of the reference's block
numbering, 3 entries per row). Prints the event-timed rates (GPU box only)."""
import os
import sys

import numpy as np
import torch  # noqa: F401  (the HIP runtime first, as bench.py)

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "p-a_multigrids_amd"))
import pamg  # noqa: E402

REPS = int(sys.argv[1]) if len(sys.argv) > 1 else 20
mesh = pamg.Mesh.read(os.path.join(ROOT, "tests", "meshes", "untitled8192.msh"))
s = pamg.SemiImplicitIterative(mesh, 5, 1, arith=1)
s.begin_timestep()
for asm in (False, True):
    ms, by = s.sweep_bench(REPS, asm)
    print(f"{'k_sweep_assembled' if asm else 'k_sweep_stencil'}: {ms:.4f} ms, {by / 1e9:.3f} GB, "
          f"{by / ms / 1e6:.1f} GB/s = {by / ms / 1e6 / 8000:.3f} of 8 TB/s", flush=True)
nrows = 3 * mesh.U * 4 ** 5
base = 3 * (np.arange(nrows, dtype=np.int32) // 3)
jloc = (base[:, None] + np.arange(1, 4, dtype=np.int32)[None, :]).reshape(-1)
sp = pamg.Sparse(s, np.arange(1, 3 * nrows, 3, dtype=np.int32), jloc,
                 np.random.default_rng(20251015).uniform(-1, 1, 3 * nrows))
ms = sp.bench(nrows, REPS)
print(f"k_csr_mul_array: {ms:.4f} ms, {52.0 * nrows / 1e9:.3f} GB, {52.0 * nrows / ms / 1e6:.1f} GB/s = "
      f"{52.0 * nrows / ms / 1e6 / 8000:.3f} of 8 TB/s", flush=True)
sp.close()
s.close()
