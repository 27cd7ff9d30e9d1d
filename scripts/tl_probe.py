"""Reference-shaped time loop (pamg_run(50, 2)) on untitled8192 at n_split 3 and 4 (k_vc_res)
and 5 (k_vc_resb): V-cycles/s with the whole run in one resident launch and, with
PAMG_NO_RESIDENT_RUN=1 in the environment, one resident launch per time step."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "p-a_multigrids_amd"))
import pamg  # noqa: E402

mesh = pamg.Mesh.read(os.path.join(ROOT, "tests", "meshes", "untitled8192.msh"))
tag = "launch per step" if os.environ.get("PAMG_NO_RESIDENT_RUN") else "one launch"
for S, L in ((3, 3), (4, 3), (5, 2), (5, 3)):
    s = pamg.SemiImplicitIterative(mesh, S, L, n_smooth=4, solver=3, arith=1, fused=3)
    s.run(20, 2)
    s.synchronize()
    best = 0.0
    for _ in range(3):
        t0 = time.perf_counter()
        s.run(50, 2)
        s.synchronize()
        best = max(best, 100 / (time.perf_counter() - t0))
    print(f"S={S} L={L} time loop 50 x 2 ({tag}): {best:10.1f} V-cycles/s", flush=True)
    s.close()
