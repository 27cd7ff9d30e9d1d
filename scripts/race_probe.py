"""Repeat test_partitioned_run_matches_single_gpu[5-8-3-0] and report where partitions and the
single domain disagree (array, partition, un_ele, face, rows), and whether either side varies
between repeats of the same run. Usage: python scripts/race_probe.py [repeats] [schedule]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "p-a_multigrids_amd"))
import pamg  # noqa: E402
from pamg.solver import halo_loopback  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 4
sched = int(sys.argv[2]) if len(sys.argv) > 2 else 0
S, nparts = 5, 8
mesh = pamg.Mesh.read(os.path.join(ROOT, "tests", "meshes", "untitled8192.msh"))
owner = mesh.x_strip_owner(nparts)
prev_full, prev_parts = None, None
for it in range(reps):
    full = pamg.SemiImplicitIterative(mesh, S, 3)
    full.run(1, 3)
    fo = full.overlap()
    fs = full.state()
    parts = [pamg.SemiImplicitIterative(mesh, S, 3, comm=(nparts, r, None, owner), fused=3, halo_exchange=0)
             for r in range(nparts)]
    if sched:
        for p in parts:
            p.set_call_schedule(sched)
    for p in parts:
        p.run(1, 3)
    halo_loopback(parts, 1)
    po = [p.overlap() for p in parts]
    ps = [p.state() for p in parts]
    nbad = 0
    for r in range(nparts):
        own = np.flatnonzero(owner == r)
        for k in fs:
            d = ps[r][k] != fs[k][:, :, own]
            if d.any():
                nbad += 1
                print(f"rep {it} part {r} state {k}: {int(d.sum())} differ", flush=True)
        for name, x, y in zip(("tov", "tovo"), po[r], fo):
            yy = y[:, :, own]
            d = x != yy
            if d.any():
                nbad += 1
                fe = np.argwhere(d.any(axis=0))
                print(f"rep {it} part {r} {name}: {int(d.sum())} differ in {len(fe)} (face, local ele) slots", flush=True)
                for f, e in fe[:12]:
                    g = own[e]
                    rows = np.flatnonzero(d[:, f, e])
                    print(f"   face {f} ele {g} (local {e}) rows {rows.min()}..{rows.max()} "
                          f"({len(rows)}) part {x[rows[0], f, e]:.6e} full {yy[rows[0], f, e]:.6e}", flush=True)
    if prev_full is not None:
        for name, a, b in zip(("tov", "tovo"), fo, prev_full):
            if (a != b).any():
                print(f"rep {it}: FULL {name} differs from the previous repeat in {int((a != b).sum())}", flush=True)
        for r in range(nparts):
            for name, a, b in zip(("tov", "tovo"), po[r], prev_parts[r]):
                if (a != b).any():
                    print(f"rep {it}: PART {r} {name} differs from the previous repeat in {int((a != b).sum())}", flush=True)
    prev_full, prev_parts = fo, po
    print(f"rep {it}: {nbad} mismatching arrays", flush=True)
    full.close()
    for p in parts:
        p.close()
