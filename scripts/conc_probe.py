"""Fused V-cycle: sequential (fused = 1) vs concurrent (fused = 2) launches of the
coarse-level and level-1 kernels; wall time per cycle without and with per-kernel
HIP events (GPU box only). Args: S,L,ns cases (default 5,3,4 3,3,4)."""
import os
import sys
import time

import torch  # noqa: F401  (binds the HIP runtime first)

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "p-a_multigrids_amd"))
import pamg  # noqa: E402

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
mesh = pamg.Mesh.read(os.path.join(ROOT, "tests", "meshes", "untitled8192.msh"))
cases = [tuple(int(x) for x in c.split(",")) for c in (sys.argv[1:] or ["5,3,4", "3,3,4"])]
for S, L, ns in cases:
    for rep in range(1):
        for fused, arith in ((1, 0), (3, 0), (1, 1), (2, 1), (3, 1)):
            s = pamg.SemiImplicitIterative(mesh, S, L, n_smooth=ns, solver=3, fused=fused, arith=arith)
            s.begin_timestep()
            s.vcycle(5)
            s.synchronize()
            n = 50 if S >= 5 else 400
            t0 = time.perf_counter()
            s.vcycle(n)
            s.synchronize()
            wall = (time.perf_counter() - t0) / n * 1e3
            s.timing_enable(0xF7F)
            s.timing_reset()
            t0 = time.perf_counter()
            s.vcycle(n)
            s.synchronize()
            wall_ev = (time.perf_counter() - t0) / n * 1e3
            tm = s.timing()
            k = {kk: round(v["ms"] / v["launches"], 4) for kk, v in tm.items() if v["launches"]}
            print(f"S={S} L={L} ns={ns} fused={fused} arith={arith}: {wall:.4f} ms/cycle ({1e3 / wall:.0f}/s), "
                  f"with events {wall_ev:.4f}; per launch {k}", flush=True)
            s.close()
