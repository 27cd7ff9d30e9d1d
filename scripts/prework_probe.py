"""What the work before the warm-up does to the driver's timed call, at N = 1 and at one rank's
partition of N = 8 (rank 0, detached: no RCCL; GPU box only). Per variant, a fresh handle, then:
  idle: begin_timestep, 5-cycle warm-up, one 20-cycle call (bench.py's timed call)
  tl:   bench.py's time-loop measurement first (run(10, 2), run(50, 2) twice), then the same
  long: pamg_run(50, 2) calls for >= 150 ms first, then the same
Alternating, 4 repetitions; ms per cycle of the 20-cycle call."""
import os
import statistics
import sys
import time

import torch  # noqa: F401

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "p-a_multigrids_amd"))
import pamg  # noqa: E402

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
mesh = pamg.Mesh.read(os.path.join(ROOT, "tests", "meshes", "untitled8192.msh"))


def one(n, variant):
    comm = None if n == 1 else (n, 0, None, mesh.x_strip_owner(n))
    s = pamg.SemiImplicitIterative(mesh, 5, 3, n_smooth=4, solver=3, comm=comm, arith=1, fused=3)
    s.begin_timestep()
    s.synchronize()
    pre = 0.0
    t0 = time.perf_counter()
    if variant == "tl":
        s.run(10, 2)
        s.run(50, 2)
        s.run(50, 2)
    elif variant == "long":
        while time.perf_counter() - t0 < 0.15:
            s.run(50, 2)
            s.synchronize()
    s.synchronize()
    pre = time.perf_counter() - t0
    s.vcycle(5)
    s.synchronize()
    s.timing_enable(0x7F7F if n == 1 else 0)
    s.timing_stride(10)
    s.timing_reset()
    t0 = time.perf_counter()
    s.vcycle(20)
    s.synchronize()
    dt = (time.perf_counter() - t0) / 20 * 1e3
    s.close()
    return dt, pre


for n in (1, 8):
    res = {v: [] for v in ("idle", "tl", "long")}
    for rep in range(4):
        for v in res:
            dt, pre = one(n, v)
            res[v].append(dt)
            print(f"N={n} rep {rep} {v:5s}: {dt:.4f} ms/cycle after {pre * 1e3:.1f} ms of pre-work", flush=True)
    for v, xs in res.items():
        print(f"N={n} {v:5s} median {statistics.median(xs):.4f} ms/cycle  all {[round(x, 4) for x in xs]}", flush=True)
