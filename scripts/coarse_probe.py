"""Sensitivity of the resident call to the coarsest level's chain: V-cycles/s and fp64 rate at
n_coarse = 15 (the reference's), 8, 4, 1 on bench.py's workload (diagnostic: other n_coarse values
are not the reference's cycle). Usage: python scripts/coarse_probe.py"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "p-a_multigrids_amd"))
import pamg  # noqa: E402

mesh = pamg.Mesh.read(os.path.join(ROOT, "tests", "meshes", "untitled8192.msh"))
for nc in (15, 8, 4, 1):
    s = pamg.SemiImplicitIterative(mesh, 5, 3, n_smooth=4, solver=3, arith=1, fused=3, n_coarse=nc)
    s.begin_timestep()
    s.vcycle(200)
    s.synchronize()
    t0 = time.perf_counter()
    s.vcycle(200)
    s.synchronize()
    dt = (time.perf_counter() - t0) / 200
    fl = s.vcycle_flops()
    print(f"n_coarse={nc:2d}: {1 / dt:9.1f} V-cycles/s, {dt * 1e3:.4f} ms/cycle, {fl / 1e9:.3f} GFLOP/cycle, "
          f"{fl / dt / 1e12:.2f} TFLOP/s", flush=True)
    s.close()
