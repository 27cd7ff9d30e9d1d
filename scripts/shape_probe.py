"""The driver's bench shape (a fresh handle, begin_timestep, a 5-cycle warm-up, one timed 20-cycle call)
under variants of what precedes it and of the timing instrumentation (GPU box only):
  fresh_ev    as bench.py r04: HIP event pair around the timed call (timing classes on)
  fresh       no events in the timed region
  sweep_ev    the level-1 HBM sweep roofline (k_sweep_assembled, `--pre` launches) right before the
              warm-up, events on
  sweep       the same without events
Each variant runs after `--idle` seconds without GPU work, in rotating order, `--reps` times; prints the
per-cycle time of every timed call and the medians."""
import argparse
import os
import sys
import time

import torch  # noqa: F401

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "p-a_multigrids_amd"))
import pamg  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--idle", type=float, default=3.0)
ap.add_argument("--pre", type=int, default=100)
a = ap.parse_args()

mesh = pamg.Mesh.read(os.path.join(ROOT, "tests", "meshes", "untitled8192.msh"))
ALL = 0x7F7F


def one(kind):
    s = pamg.SemiImplicitIterative(mesh, 5, 3, n_smooth=4, solver=3, arith=1, fused=3)
    s.begin_timestep()
    s.synchronize()
    time.sleep(a.idle)
    pre_ms = 0.0
    if kind.startswith("sweep"):
        ms, _ = s.sweep_bench(a.pre, True)
        pre_ms = ms * a.pre
    s.vcycle(5)
    s.synchronize()
    ev = kind.endswith("_ev")
    s.timing_enable(ALL if ev else 0)
    s.timing_stride(10)
    s.timing_reset()
    s.synchronize()
    t0 = time.perf_counter()
    s.vcycle(20)
    s.synchronize()
    dt = (time.perf_counter() - t0) / 20 * 1e3
    kms = None
    if ev:
        k = s.timing()["vcycle_res"]
        kms = k["ms"] / max(1, k["launches"]) / 20
    s.close()
    return dt, kms, pre_ms


kinds = ["fresh_ev", "fresh", "sweep_ev", "sweep"]
res = {k: [] for k in kinds}
for r in range(a.reps):
    for i in range(len(kinds)):
        k = kinds[(i + r) % len(kinds)]
        dt, kms, pre = one(k)
        res[k].append(dt)
        print(f"rep {r} {k:9s}: {dt:.4f} ms/cycle" + (f" (kernel {kms:.4f})" if kms else "") +
              (f" after {pre:.1f} ms of sweeps" if pre else ""), flush=True)
for k in kinds:
    v = sorted(res[k])
    print(f"{k:9s} median {v[len(v) // 2]:.4f} ms/cycle = {1 / v[len(v) // 2] * 1e3:.0f} V-cycles/s  all {v}", flush=True)
