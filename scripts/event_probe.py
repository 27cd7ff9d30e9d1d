"""Wall time per V-cycle of one 50-cycle call with the library's HIP-event timing off and on
(bench.py's stride), same box; GPU box only. Shows what the sampled events cost the bench."""
import os
import sys
import time

import torch  # noqa: F401

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "p-a_multigrids_amd"))
import pamg  # noqa: E402

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
mesh = pamg.Mesh.read(os.path.join(ROOT, "tests", "meshes", "untitled8192.msh"))
s = pamg.SemiImplicitIterative(mesh, 5, 3, n_smooth=4, solver=3, fused=3, arith=1)
s.begin_timestep()
s.vcycle(5)
s.synchronize()
for rep in range(3):
    for mask, stride in ((0, 10), (0xF7F, 10), (0xF7F, 1000000)):
        s.timing_enable(mask)
        s.timing_stride(stride)
        s.timing_reset()
        s.synchronize()
        t0 = time.perf_counter()
        s.vcycle(50)
        s.synchronize()
        dt = (time.perf_counter() - t0) / 50 * 1e3
        tm = s.timing()
        ev = {k: round(v["ms"] / v["launches"], 4) for k, v in tm.items() if v["launches"]}
        print(f"mask={mask:#x} stride={stride}: {dt:.4f} ms/cycle  events {ev}", flush=True)
s.close()
