"""Per-field relative error of the contracted arithmetic (arith = 1) against the
reference's fp64 goldens, with the cancellation factor max|RHS_l| / max|res_l| of
the reference's own residuals (GPU box only)."""
import os
import sys

import numpy as np
import torch  # noqa: F401

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "p-a_multigrids_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import goldens  # noqa: E402
import pamg  # noqa: E402

for name in goldens.names():
    meta, d = goldens.load(name)
    if meta["precision"] != "fp64" or meta["solver"] == 2:
        continue
    m = pamg.Mesh.read(os.path.join(goldens.MESHES, meta["mesh"]))
    s = pamg.SemiImplicitIterative(m, meta["n_split"], meta["levels"], n_smooth=meta["n_smooth"],
                                   solver=meta["solver"], arith=1)
    s.run(meta["ntime"], meta["n_multigrid"])
    st = s.state()
    st["t_overlap"], st["t_overlap_old"] = s.overlap()
    errs = {}
    for k, v in st.items():
        try:
            errs[k] = goldens.rel_err(v, d[k]) if k in d else goldens.compare_sampled(d, k, v)
        except KeyError:
            continue
    kap = {}
    for l in range(1, meta["levels"] + 1):
        if f"RHS_L{l}" in d and f"res_L{l}" in d:
            kap[l] = float(np.abs(d[f"RHS_L{l}"]).max() / max(np.abs(d[f"res_L{l}"]).max(), 1e-300))
    print(name, {k: f"{e:.1e}" for k, e in errs.items()}, "kappa", {k: f"{v:.1e}" for k, v in kap.items()},
          flush=True)
