"""Per-rank cycle time of the x-strip partition of untitled8192 at N = 1, 2, 4, 8 ranks,
simulated on one GPU (rank 0's partition, detached: no RCCL), to size the strong-scaling
overheads (GPU box only)."""
import os
import sys
import time

import torch  # noqa: F401

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "p-a_multigrids_amd"))
import pamg  # noqa: E402

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
S = int(sys.argv[1]) if len(sys.argv) > 1 else 5
FUSED = int(sys.argv[2]) if len(sys.argv) > 2 else 3
MESH = sys.argv[3] if len(sys.argv) > 3 else "untitled8192.msh"
mesh = pamg.Mesh.read(os.path.join(ROOT, "tests", "meshes", MESH))
base = None
for n in (1, 2, 4, 8):
    comm = None if n == 1 else (n, 0, None, mesh.x_strip_owner(n))
    s = pamg.SemiImplicitIterative(mesh, S, 3, n_smooth=4, solver=3, comm=comm, arith=1, fused=FUSED)
    s.begin_timestep()
    s.vcycle(200)   # settle the clocks (bench.py's default warm-up)
    s.synchronize()
    res = []
    for timed in (0, 1):
        s.timing_enable(0x3F7F if timed else 0)
        s.timing_reset()
        k = 200
        t0 = time.perf_counter()
        s.vcycle(k)
        s.synchronize()
        dt = (time.perf_counter() - t0) / k * 1e3
        tm = s.timing()
        res.append((dt, {kk: round(v["ms"] / k, 4) for kk, v in tm.items() if v["launches"]}))
    t0 = time.perf_counter()
    s.vcycle(20)   # the driver's call length
    s.synchronize()
    d20 = (time.perf_counter() - t0) / 20 * 1e3
    if base is None:
        base = res[0][0]
    print(f"{MESH} S={S} fused={FUSED} N={n} (rank 0: {s.U} un_eles): {res[0][0]:.4f} ms/cycle (ideal {base / n:.4f}, eff {base / n / res[0][0]:.2f}); "
          f"20-cycle call {d20:.4f} ms/cycle; timed {res[1][0]:.4f} {res[1][1]}; rank fp64 "
          f"{s.vcycle_flops() / (res[0][0] * 1e-3) / 1e12 / 78.6:.3f} of peak", flush=True)
    s.close()
