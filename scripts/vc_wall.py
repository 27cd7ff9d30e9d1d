"""Wall time per fused V-cycle with and without the per-kernel timing events (GPU box only)."""
import os
import sys
import time

import torch  # noqa: F401

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "p-a_multigrids_amd"))
import pamg  # noqa: E402

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
mesh = pamg.Mesh.read(os.path.join(ROOT, "tests", "meshes", "untitled8192.msh"))
S = int(sys.argv[1]) if len(sys.argv) > 1 else 5
s = pamg.SemiImplicitIterative(mesh, S, 3, n_smooth=4, solver=3)
s.begin_timestep()
s.vcycle(5)
s.synchronize()
for timed in (0, 1, 0, 1):
    s.timing_enable(0xF7F if timed else 0)
    s.timing_reset()
    n = 50
    t0 = time.perf_counter()
    s.vcycle(n)
    s.synchronize()
    dt = (time.perf_counter() - t0) / n * 1e3
    tm = s.timing()
    k = {kk: round(v["ms"] / n, 4) for kk, v in tm.items() if v["launches"]}
    print(f"S={S} timing={timed}: {dt:.4f} ms/cycle {k}", flush=True)
s.close()
