"""The reference-shaped time loop (pamg_run: ntime steps of begin_timestep + n_multigrid
V-cycles) on untitled8192 at n_split = 5: wall time per step; run under rocprofv3
--kernel-trace --stats for the per-kernel split (GPU box only)."""
import os
import sys
import time

import torch  # noqa: F401

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "p-a_multigrids_amd"))
import pamg  # noqa: E402

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
mesh = pamg.Mesh.read(os.path.join(ROOT, "tests", "meshes", "untitled8192.msh"))
s = pamg.SemiImplicitIterative(mesh, 5, 3, n_smooth=4, solver=3, fused=3, arith=1)
s.run(20, 2)   # warm-up
s.synchronize()
t0 = time.perf_counter()
s.run(50, 2)
s.synchronize()
dt = (time.perf_counter() - t0) / 50
print(f"time loop: {dt * 1e3:.4f} ms per step of 2 V-cycles, {2 / dt:.1f} V-cycles/s", flush=True)
s.close()
