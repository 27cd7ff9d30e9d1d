"""Phase timeline of the fused V-cycle kernel from its in-kernel stamps
(PAMG_VCYCLE_STAMPS), GPU box only. usage: stamp_probe.py S L [ns nc [N]]"""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
if os.environ.get("PAMG_VCYCLE_STAMPS") is None:
    out = os.path.join(os.environ.get("TMPDIR", "/tmp"), "pamg_stamps.bin")
    if os.path.exists(out):
        os.remove(out)
    r = subprocess.run([sys.executable, __file__] + sys.argv[1:], env=dict(os.environ, PAMG_VCYCLE_STAMPS=out))
    if r.returncode:
        sys.exit(r.returncode)
    raw = np.fromfile(out, dtype=np.int64)
    recs = {}
    i = 0
    while i < raw.size:
        g, w, s, L = raw[i:i + 4]
        n = g * w * s
        recs.setdefault("coarse" if L < 0 else "fine", []).append(raw[i + 4:i + 4 + n].reshape(g, w, s))
        i += 4 + n
    names = {"fine": ["prologue(+chain)+sweeps", "halo+residual", "final sweeps", "stores+halo", "cascade+coarse(pipe)", "", ""],
             "coarse": ["prologue+restrict", "L2..C-1 restr-leg", "coarse chain", "prolong legs", "", "",
                        "cascade"]}
    for kind, lst in recs.items():
        # fine: the call's pipelined launches come before its last (plain) level-1 launch
        st = lst[-2] if kind == "fine" and len(lst) > 1 else lst[-1]
        t = st[:, :, :8].astype(np.float64) * 10.0 / 1000.0  # 100 MHz ticks -> us
        ok = st[:, :, 0] > 0
        t0 = t[:, :, 0][ok].min()
        span = t[:, :, 7].max() - t0
        print(f"== {kind}: launches={len(lst)} grid={st.shape[0]} waves/WG={st.shape[1]} span={span:.1f} us")
        for ph in range(7):
            if not names[kind][ph]:
                continue
            nxt = ph + 1
            while nxt < 8 and not (st[:, :, nxt] > 0).any():
                nxt += 1
            d = t[:, :, nxt] - t[:, :, ph]
            valid = (st[:, :, nxt] > 0) & (st[:, :, ph] > 0)
            d0 = d[:, 0][valid[:, 0]]
            dr = d[:, 1:][valid[:, 1:]]
            if d0.size == 0:
                continue
            line = f"{names[kind][ph]:>20s}: wave0 median {np.median(d0):6.2f} p90 {np.percentile(d0, 90):6.2f}"
            if dr.size:
                line += f" | other waves median {np.median(dr):6.2f} p90 {np.percentile(dr, 90):6.2f} us"
            print(line)
        life = t[:, :, 7].max(1) - t[:, :, 0].min(1)
        print(f"WG lifetime median {np.median(life):.2f} p10 {np.percentile(life, 10):.2f} "
              f"p90 {np.percentile(life, 90):.2f} us; mean WGs in flight per CU {life.sum() / span / 256:.2f}")
    sys.exit(0)

import torch  # noqa: E402,F401
sys.path.insert(0, os.path.join(ROOT, "p-a_multigrids_amd"))
import pamg  # noqa: E402

S, L = int(sys.argv[1]), int(sys.argv[2])
ns = int(sys.argv[3]) if len(sys.argv) > 3 else 4
nc = int(sys.argv[4]) if len(sys.argv) > 4 else 15
mesh = pamg.Mesh.read(os.path.join(ROOT, "tests", "meshes", "untitled8192.msh"))
N = int(sys.argv[5]) if len(sys.argv) > 5 else 1   # rank 0's x-strip partition of N (detached)
comm = None if N == 1 else (N, 0, None, mesh.x_strip_owner(N))
s = pamg.SemiImplicitIterative(mesh, S, L, n_smooth=ns, n_coarse=nc, solver=3, arith=1, fused=3, comm=comm)
s.begin_timestep()
s.vcycle(100 if N > 1 else 4)   # a partition's launches are small: settle the clocks first
s.synchronize()
s.close()
