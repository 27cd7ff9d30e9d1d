"""The driver's call shape over time: a fresh handle, a 5-cycle warm-up, then 20-cycle calls back
to back (each synchronized, as bench.py's timed call) for about a second of GPU time, printing the
per-cycle time of every call -- how far the first call's rate is from the settled one, and how
long the GPU takes to get there (GPU box only)."""
import os
import sys
import time

import torch  # noqa: F401

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "p-a_multigrids_amd"))
import pamg  # noqa: E402

mesh = pamg.Mesh.read(os.path.join(ROOT, "tests", "meshes", "untitled8192.msh"))
s = pamg.SemiImplicitIterative(mesh, 5, 3, n_smooth=4, solver=3, arith=1, fused=3)
s.begin_timestep()
s.vcycle(5)
s.synchronize()
t_start = time.perf_counter()
rows = []
for i in range(1000):
    t0 = time.perf_counter()
    s.vcycle(20)
    s.synchronize()
    t1 = time.perf_counter()
    rows.append((t0 - t_start, (t1 - t0) / 20 * 1e3))
for i in list(range(0, 20)) + list(range(20, 1000, 40)):
    print(f"call {i:4d} at {1e3 * rows[i][0]:8.2f} ms: {rows[i][1]:.4f} ms/cycle", flush=True)
last = sorted(r[1] for r in rows[-100:])
print(f"first call {rows[0][1]:.4f}; median of the last 100 calls {last[50]:.4f} ms/cycle "
      f"(first / settled = {rows[0][1] / last[50]:.3f})", flush=True)
s.close()
