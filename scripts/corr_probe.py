"""The corrected V-cycle (cycle = 1) on bench.py's workload: the resident call's V-cycles/s and fp64
rate (bench.py measure_corrected), per-step beside it, and a bitwise check of the resident state against
the per-step sequence after a 5-cycle call.
Usage: python scripts/corr_probe.py [n_split] [levels] [cycles]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "p-a_multigrids_amd"))
import pamg  # noqa: E402
import bench  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 5
L = int(sys.argv[2]) if len(sys.argv) > 2 else 3
N = int(sys.argv[3]) if len(sys.argv) > 3 else 200
mesh = pamg.Mesh.read(os.path.join(ROOT, "tests", "meshes", "untitled8192.msh"))
print(bench.measure_corrected(pamg, mesh, S, L, 4, 1, 0, N), flush=True)
st = []
for fused in (3, 0):
    s = pamg.SemiImplicitIterative(mesh, S, L, n_smooth=4, solver=3, arith=1, cycle=1, fused=fused)
    s.begin_timestep()
    s.vcycle(5)
    st.append((s.state(), s.overlap()))
    s.close()
same = all(np.array_equal(st[0][0][k], st[1][0][k]) for k in st[1][0]) and \
    all(np.array_equal(x, y) for x, y in zip(st[0][1], st[1][1]))
r = float(np.abs(st[0][0]["res_L1"]).max())
print(f"resident == per-step bitwise: {same}; max|res_L1| after 5 cycles {r:.3e}", flush=True)
