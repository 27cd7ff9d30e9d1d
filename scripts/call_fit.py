"""Kernel time of the resident call against its cycle count (GPU box only): a warmed handle (bench.py's
workload, 400 cycles of warm-up), then calls of n = 1, 2, 5, 10, 20, 50, 100, 200 cycles, each timed by its
HIP event pair, `--reps` times in rotating order; the median per n and a least-squares line t = a + b n over
them -- a is the per-call fixed part inside the launch (tile loads / stores per round, the last round's tail),
b the per-cycle cost."""
import argparse
import os
import sys

import numpy as np
import torch  # noqa: F401

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "p-a_multigrids_amd"))
import pamg  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--nsplit", type=int, default=5)
a = ap.parse_args()
mesh = pamg.Mesh.read(os.path.join(ROOT, "tests", "meshes", "untitled8192.msh"))
s = pamg.SemiImplicitIterative(mesh, a.nsplit, 3, n_smooth=4, solver=3, arith=1, fused=3)
s.begin_timestep()
s.vcycle(400)
s.synchronize()
ns = [1, 2, 5, 10, 20, 50, 100, 200]
res = {n: [] for n in ns}
for r in range(a.reps):
    for i in range(len(ns)):
        n = ns[(i + r) % len(ns)]
        s.timing_enable(1 << 12)
        s.timing_stride(1)
        s.timing_reset()
        s.vcycle(n)
        s.synchronize()
        k = s.timing()["vcycle_res"]
        res[n].append(k["ms"] / max(1, k["launches"]))
        s.timing_enable(0)
        s.vcycle(20)   # keep the clocks up between the timed calls
        s.synchronize()
med = np.array([np.median(res[n]) for n in ns])
A = np.vstack([np.ones(len(ns)), ns]).T
(a0, b0), *_ = np.linalg.lstsq(A, med, rcond=None)
for n, m in zip(ns, med):
    print(f"n={n:4d}: {m:.4f} ms per call, {m / n * 1e3:.2f} us per cycle (all {['%.4f' % v for v in res[n]]})", flush=True)
print(f"fit: {a0 * 1e3:.1f} us per call + {b0 * 1e3:.2f} us per cycle (n_split {a.nsplit})")
s.close()
