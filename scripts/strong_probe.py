"""Per-rank cycle time of the x-strip partition of untitled8192 at N = 1, 2, 4, 8 ranks,
simulated on one GPU (rank 0's partition, detached: no RCCL), to size the strong-scaling
overheads (GPU box only).

Per N: the steady state (a 200-cycle call after a 200-cycle warm-up, with and without the
per-kernel events), then the driver's call the way bench.py times it -- a fresh handle, a
5-cycle warm-up, one 20-cycle call (events on at N = 1 only, as bench.py: live events on one
GPU, none on N ranks) -- and the median / min of 15 more such calls. The last column is the
driver-shape ratio value_N / value_1 (bench.py's value: the whole mesh's 20 cycles over the
rank's call time)."""
import os
import statistics
import sys
import time

import torch  # noqa: F401

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "p-a_multigrids_amd"))
import pamg  # noqa: E402

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
S = int(sys.argv[1]) if len(sys.argv) > 1 else 5
FUSED = int(sys.argv[2]) if len(sys.argv) > 2 else 3
MESH = sys.argv[3] if len(sys.argv) > 3 else "untitled8192.msh"
ALL_CLASSES, EVENT_STRIDE = 0x7F7F, 10   # bench.py's
mesh = pamg.Mesh.read(os.path.join(ROOT, "tests", "meshes", MESH))


def handle(n):
    comm = None if n == 1 else (n, 0, None, mesh.x_strip_owner(n))
    return pamg.SemiImplicitIterative(mesh, S, 3, n_smooth=4, solver=3, comm=comm, arith=1, fused=FUSED)


def call20(s, n):
    """one 20-cycle call timed as bench.py times it (ms per cycle)"""
    s.timing_enable(ALL_CLASSES if n == 1 else 0)
    s.timing_stride(EVENT_STRIDE)
    s.timing_reset()
    s.synchronize()
    t0 = time.perf_counter()
    s.vcycle(20)
    s.synchronize()
    return (time.perf_counter() - t0) / 20 * 1e3


base = None
drv1 = None
for n in (1, 2, 4, 8):
    # the driver's shape first, on a fresh handle: 5-cycle warm-up, one timed 20-cycle call
    s = handle(n)
    s.begin_timestep()
    s.vcycle(5)
    s.synchronize()
    first = call20(s, n)
    reps = sorted(call20(s, n) for _ in range(15))
    med, mn = statistics.median(reps), reps[0]
    # then the steady state
    s.timing_enable(0)
    s.vcycle(200)
    s.synchronize()
    res = []
    for timed in (0, 1):
        s.timing_enable(0x3F7F if timed else 0)
        s.timing_stride(1)
        s.timing_reset()
        k = 200
        t0 = time.perf_counter()
        s.vcycle(k)
        s.synchronize()
        dt = (time.perf_counter() - t0) / k * 1e3
        tm = s.timing()
        res.append((dt, {kk: round(v["ms"] / k, 4) for kk, v in tm.items() if v["launches"]}))
    if base is None:
        base, drv1 = res[0][0], (first, med)
    print(f"{MESH} S={S} fused={FUSED} N={n} (rank 0: {s.U} un_eles): 200-cycle {res[0][0]:.4f} ms/cycle "
          f"(ideal {base / n:.4f}, eff {base / n / res[0][0]:.2f}; timed {res[1][0]:.4f} {res[1][1]}); "
          f"driver shape: first 20-cycle call {first:.4f} ms/cycle, 15 more median {med:.4f} min {mn:.4f}; "
          f"value_N / value_1 = {drv1[0] / first:.2f} (first calls), {drv1[1] / med:.2f} (medians); rank fp64 "
          f"{s.vcycle_flops() / (res[0][0] * 1e-3) / 1e12 / 78.6:.3f} of peak", flush=True)
    s.close()
