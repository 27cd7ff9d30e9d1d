"""Timing probe of the fused V-cycle kernel vs the per-step kernel sequence
over (n_split, levels, n_smooth, n_coarse) variants (GPU box only)."""
import os
import sys
import time

import torch  # noqa: F401  (binds the HIP runtime first)

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "p-a_multigrids_amd"))
import pamg  # noqa: E402

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
mesh = pamg.Mesh.read(os.path.join(ROOT, "tests", "meshes", "untitled8192.msh"))
cases = [(5, 3, 4, 15), (5, 3, 4, 1), (5, 3, 1, 15), (5, 3, 1, 1), (5, 1, 4, 15), (5, 1, 4, 1), (5, 2, 4, 15),
         (5, 4, 4, 15), (4, 3, 4, 15), (3, 3, 4, 15)]
if len(sys.argv) > 1:
    cases = [tuple(int(x) for x in c.split(",")) for c in sys.argv[1:]]
for S, L, ns, nc in cases:
    row = []
    for fused in (1, 0):
        s = pamg.SemiImplicitIterative(mesh, S, L, n_smooth=ns, solver=3, fused=fused, n_coarse=nc)
        s.begin_timestep()
        s.vcycle(3)
        s.synchronize()
        s.timing_enable(0xF7F)
        s.timing_reset()
        n = 20
        t0 = time.perf_counter()
        s.vcycle(n)
        s.synchronize()
        dt = (time.perf_counter() - t0) / n * 1e3
        tm = s.timing()
        k = {kk: round(v["ms"] / n, 4) for kk, v in tm.items() if v["launches"]}
        row.append((round(dt, 4), k))
        s.close()
    print(f"S={S} L={L} ns={ns} nc={nc}: fused {row[0][0]} ms {row[0][1]} | unfused {row[1][0]} ms {row[1][1]}",
          flush=True)
