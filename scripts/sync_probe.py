"""Wall time of the driver's 20-cycle call (vcycle(20) + synchronize) per rank partition of
untitled8192 S=5, simulated on one GPU (detached, rank 0); GPU box only. archive/profiles/r03_m_sync_probe.txt is its
A/B of the host wait (mode 0 spin, 1 hipStreamSynchronize, 2 sleeping poll) under a switch
since removed (the waits measured within noise)."""
import os
import statistics
import sys
import time

import torch  # noqa: F401

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "p-a_multigrids_amd"))
import pamg  # noqa: E402

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
mesh = pamg.Mesh.read(os.path.join(ROOT, "tests", "meshes", "untitled8192.msh"))
for n in (1, 8):
    comm = None if n == 1 else (n, 0, None, mesh.x_strip_owner(n))
    s = pamg.SemiImplicitIterative(mesh, 5, 3, n_smooth=4, solver=3, comm=comm, arith=1, fused=3)
    s.begin_timestep()
    s.vcycle(200)
    s.synchronize()
    k200 = []
    for _ in range(3):
        t0 = time.perf_counter()
        s.vcycle(200)
        s.synchronize()
        k200.append((time.perf_counter() - t0) / 200 * 1e3)
    w = []
    for _ in range(40):
        t0 = time.perf_counter()
        s.vcycle(20)
        s.synchronize()
        w.append((time.perf_counter() - t0) * 1e3)
    c1 = min(k200)
    print(f"N={n}: 200-cycle {c1:.4f} ms/cycle; 20-cycle call median {statistics.median(w):.4f} ms "
          f"min {min(w):.4f} ms -> {statistics.median(w) / 20:.4f} ms/cycle; fixed ~{(statistics.median(w) - 20 * c1) * 1e3:.1f} us", flush=True)
    s.close()
