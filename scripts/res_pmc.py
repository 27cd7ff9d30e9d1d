"""One warm-up and one timed 200-cycle resident call on bench.py's workload, for rocprofv3 PMC
passes (scripts/full_check.sh style): python scripts/res_pmc.py [cycles]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "p-a_multigrids_amd"))
import pamg  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 200
mesh = pamg.Mesh.read(os.path.join(ROOT, "tests", "meshes", "untitled8192.msh"))
s = pamg.SemiImplicitIterative(mesh, 5, 3, n_smooth=4, solver=3, arith=1, fused=3)
s.begin_timestep()
s.vcycle(n)
s.synchronize()
t0 = time.perf_counter()
s.vcycle(n)
s.synchronize()
dt = time.perf_counter() - t0
print(f"{n / dt:.1f} V-cycles/s, {s.vcycle_flops() * n / dt / 1e12:.2f} TFLOP/s fp64", flush=True)
s.close()
