"""A/B wall time per V-cycle of one library build (PAMG_LIB) for given
(n_split, levels, fused, arith) cases; GPU box only. Args: S,L,fused,arith ..."""
import os
import sys
import time

import torch  # noqa: F401

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "p-a_multigrids_amd"))
import pamg  # noqa: E402

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
mesh = pamg.Mesh.read(os.path.join(ROOT, "tests", "meshes", "untitled8192.msh"))
out = []
for c in sys.argv[1:] or ["5,3,3,1"]:
    v = [int(x) for x in c.split(",")]
    S, L, fused, arith = v[:4]
    N = v[4] if len(v) > 4 else 1   # rank 0's x-strip partition of N (detached, no exchange)
    comm = None if N == 1 else (N, 0, None, mesh.x_strip_owner(N))
    s = pamg.SemiImplicitIterative(mesh, S, L, n_smooth=4, solver=3, fused=fused, arith=arith, comm=comm)
    s.begin_timestep()
    s.vcycle(5)
    s.synchronize()
    n = 100 if S >= 5 else 500
    best = 1e9
    for _ in range(3):
        t0 = time.perf_counter()
        s.vcycle(n)
        s.synchronize()
        best = min(best, (time.perf_counter() - t0) / n * 1e3)
    out.append(f"{c}: {best:.4f} ms")
    s.close()
print(" | ".join(out), flush=True)
