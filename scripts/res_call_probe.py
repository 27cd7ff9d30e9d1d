"""Kernel time of bench.py's resident call at n = 20 (the driver's call) and n = 200 on a warmed handle,
HIP event pair per call, medians of `--reps` (GPU box only; A/B of PAMG_* settings run per process)."""
import argparse
import os
import sys

import numpy as np
import torch  # noqa: F401

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "p-a_multigrids_amd"))
import pamg  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=8)
ap.add_argument("--tag", default="")
a = ap.parse_args()
mesh = pamg.Mesh.read(os.path.join(ROOT, "tests", "meshes", "untitled8192.msh"))
s = pamg.SemiImplicitIterative(mesh, 5, 3, n_smooth=4, solver=3, arith=1, fused=3)
s.begin_timestep()
s.vcycle(400)
s.synchronize()
out = {}
for n, reps in ((20, a.reps), (200, max(2, a.reps // 3))):
    v = []
    for _ in range(reps):
        s.timing_enable(1 << 12)
        s.timing_stride(1)
        s.timing_reset()
        s.vcycle(n)
        s.synchronize()
        k = s.timing()["vcycle_res"]
        v.append(k["ms"] / max(1, k["launches"]))
    out[n] = float(np.median(v))
print(f"{a.tag}: n=20 {out[20]:.4f} ms ({out[20] / 20 * 1e3:.2f} us/cycle), n=200 {out[200]:.4f} ms "
      f"({out[200] / 200 * 1e3:.2f} us/cycle)", flush=True)
s.close()
