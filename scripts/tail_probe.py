"""Per-rank cycle time of rank 0's x-strip partition at N = 8 (simulated on one GPU) for
variants of the coarse work: L = 3 (n_coarse 15 / 1), L = 2, L = 1 (GPU box only)."""
import os
import sys
import time

import torch  # noqa: F401

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "p-a_multigrids_amd"))
import pamg  # noqa: E402

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
mesh = pamg.Mesh.read(os.path.join(ROOT, "tests", "meshes", "untitled8192.msh"))
for n in (1, 8):
    for L, nc in ((3, 15), (3, 1), (2, 15), (1, 15)):
        comm = None if n == 1 else (n, 0, None, mesh.x_strip_owner(n))
        s = pamg.SemiImplicitIterative(mesh, 5, L, n_smooth=4, solver=3, comm=comm, arith=1, n_coarse=nc)
        s.begin_timestep()
        s.vcycle(5)
        s.synchronize()
        best = 1e9
        for _ in range(3):
            t0 = time.perf_counter()
            s.vcycle(50)
            s.synchronize()
            best = min(best, (time.perf_counter() - t0) / 50 * 1e3)
        print(f"N={n} L={L} n_coarse={nc}: {best:.4f} ms/cycle", flush=True)
        s.close()
