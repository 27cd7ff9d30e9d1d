"""The contracted arithmetic (arith = 1, bench.py's) against the reference's operation order
(arith = 0) on bench.py's workload: untitled8192, n_split = 5, L = 3, one time step and a
20-cycle pamg_vcycle call. Both are the HIP path (each bitwise equal to the oracle's restatement
of its arithmetic, tests/test_contracted_oracle.py; arith = 0 is the reference's order). Per
level: the cancellation factor kappa_l = max|RHS_l| / max|res_l| and the max abs difference of
every field, relative to the field's own scale and to the scale of the terms it was computed
from. GPU box; the committed output is archive/profiles/r02_conditioning.txt."""
import os
import sys

import numpy as np
import torch  # noqa: F401

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "p-a_multigrids_amd"))
import pamg  # noqa: E402

CASES = [("untitled8192.msh", 5, 3, 20), ("untitled8192.msh", 3, 3, 20), ("irregular.msh", 6, 3, 20),
         ("900_ele.msh", 4, 4, 20), ("test_sn2.msh", 4, 2, 20)]
for mesh, S, L, n in CASES:
    m = pamg.Mesh.read(os.path.join(ROOT, "tests", "meshes", mesh))
    st = []
    for arith in (0, 1):
        s = pamg.SemiImplicitIterative(m, S, L, arith=arith, fused=3)
        s.begin_timestep()
        s.vcycle(n)
        st.append(s.state())
        s.close()
    a, b = st
    amax = lambda k: float(np.abs(a[k]).max())  # noqa: E731
    print(f"{mesh} n_split={S} L={L}, one step of {n} V-cycles: arith 1 vs arith 0 (max abs diff / scale)")
    for l in range(1, L + 1):
        kap = amax(f"RHS_L{l}") / max(amax(f"res_L{l}"), 1e-300)
        row = [f"  L{l}: kappa {kap:9.2e}"]
        for k in (f"tnew_L{l}", f"RHS_L{l}", f"res_L{l}"):
            d = float(np.abs(a[k] - b[k]).max())
            row.append(f"{k.split('_')[0]} {d / max(amax(k), 1e-300):8.1e}")
        row.append(f"res/max|RHS_{l}| {float(np.abs(a[f'res_L{l}'] - b[f'res_L{l}']).max()) / amax(f'RHS_L{l}'):8.1e}")
        if l >= 2:
            row.append(f"RHS/max|RHS_{l - 1}| {float(np.abs(a[f'RHS_L{l}'] - b[f'RHS_L{l}']).max()) / amax(f'RHS_L{l - 1}'):8.1e}")
        # the bound of tests/test_gpu_parity.py check_contracted: 1e-12 of the level-1 scales
        e_res = float(np.abs(a[f"res_L{l}"] - b[f"res_L{l}"]).max()) / amax("RHS_L1")
        e_rhs = float(np.abs(a[f"RHS_L{l}"] - b[f"RHS_L{l}"]).max()) / amax("RHS_L1")
        e_t = float(np.abs(a[f"tnew_L{l}"] - b[f"tnew_L{l}"]).max()) / amax("tnew_L1")
        row.append(f"[res, RHS]/max|RHS_1| {e_res:8.1e} {e_rhs:8.1e}, tnew/max|tnew_1| {e_t:8.1e}")
        print(", ".join(row), flush=True)
    d = float(np.abs(a["tnew_nonlin"] - b["tnew_nonlin"]).max()) / amax("tnew_nonlin")
    print(f"  tnew_nonlin (level 1) {d:8.1e}", flush=True)
