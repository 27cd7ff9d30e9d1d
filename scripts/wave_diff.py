"""Which un_eles / positions differ between the wavefront smoother call and one launch per sweep
(level 1 of untitled8192 at n_split 5). usage: wave_diff.py [n_split] [levels] [n_smooth]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "p-a_multigrids_amd"))
import pamg  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 5
L = int(sys.argv[2]) if len(sys.argv) > 2 else 3
NS = int(sys.argv[3]) if len(sys.argv) > 3 else 4
m = pamg.Mesh.read(os.path.join(ROOT, "tests", "meshes", "untitled8192.msh"))


def run(wave):
    os.environ["PAMG_FACE_WAVE"] = "1" if wave else "0"
    g = pamg.SemiImplicitIterative(m, S, L, n_smooth=NS, solver=3, op=1)
    g.begin_timestep()
    g.smoother(1)
    g.synchronize()
    out = {k: g.get(k, 1) for k in (pamg.TNEW, pamg.TNEW_NONLIN)}
    ov = g.overlap()
    g.close()
    return out, ov


a, ova = run(True)
b, ovb = run(False)
for k in a:
    d = np.abs(a[k] - b[k])
    bad = np.argwhere(d > 0)
    print(k, a[k].shape, "mismatched", len(bad))
    if len(bad):
        us = np.unique(bad[:, 2])
        ps = np.unique(bad[:, 1])
        print("  un_eles", len(us), us[:20], " positions", len(ps), ps[:20])
for x, y, n in zip(ova, ovb, ("t_overlap", "t_overlap_old")):
    d = np.abs(x - y)
    bad = np.argwhere(d > 0)
    print(n, x.shape, "mismatched", len(bad), np.unique(bad[:, 2])[:20] if len(bad) else "")
