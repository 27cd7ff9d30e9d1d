"""Workgroup timeline of the resident call (k_vc_resb) on bench.py's workload (GPU box only): a 20-cycle call
after a warm-up, with a PAMG_STAMPS=1 build (PAMG_LIB) recording every wave's start and end; per workgroup its
life (first wave start -> last wave end), and against the launch's span how busy the workgroup slots were --
3 x CUs slots over the span, so idle slot time = dispatch gaps and the last round's tail."""
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
if os.environ.get("PAMG_VCYCLE_STAMPS") is None:
    path = os.path.join(tempfile.mkdtemp(), "res.bin")
    env = dict(os.environ, PAMG_LIB=os.path.join(ROOT, "scripts", "ablibs", "pp_stamps.so"), PAMG_VCYCLE_STAMPS=path)
    r = subprocess.run([sys.executable, __file__] + sys.argv[1:], env=env)
    if r.returncode:
        sys.exit(r.returncode)
    raw = np.fromfile(path, dtype=np.int64)
    recs = []
    i = 0
    while i < raw.size:
        g, w, ns, L = raw[i:i + 4]
        recs.append(raw[i + 4:i + 4 + g * w * ns].reshape(g, w, ns))
        i += 4 + g * w * ns
    for n, st in zip(("warm-up", "timed"), recs[-2:]):
        t0 = st[:, :, 0]
        t1 = st[:, :, 7]
        start = np.where(t0 > 0, t0, np.iinfo(np.int64).max).min(axis=1)
        end = t1.max(axis=1)
        life = (end - start) * 1e-2   # us
        span = (end.max() - start.min()) * 1e-2
        slots = 3 * 256
        print(f"{n}: {st.shape[0]} workgroups, span {span:.1f} us; workgroup life median {np.median(life):.2f} us "
              f"(min {life.min():.2f}, max {life.max():.2f}); slot occupancy {life.sum() / (slots * span):.3f}")
        rel = np.sort((start - start.min()) * 1e-2)
        hist, edges = np.histogram(rel, bins=22)
        print("   starts (us -> count): " + " ".join(f"{edges[k]:.0f}:{hist[k]}" for k in range(len(hist))))
    sys.exit(0)

sys.path.insert(0, os.path.join(ROOT, "p-a_multigrids_amd"))
import torch  # noqa: E402,F401
import pamg  # noqa: E402
mesh = pamg.Mesh.read(os.path.join(ROOT, "tests", "meshes", "untitled8192.msh"))
s = pamg.SemiImplicitIterative(mesh, 5, 3, n_smooth=4, solver=3, arith=1, fused=3)
s.begin_timestep()
s.vcycle(20)
s.vcycle(20)
s.synchronize()
s.close()
