"""Resident (schedule 3) vs one launch per cycle (schedule 1) on bench.py's workload:
bitwise state after a call and a time loop, V-cycles/s of calls of 200 and 20 cycles and of
the reference-shaped time loop (2 cycles per step). Usage: python scripts/res_probe.py [S L]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "p-a_multigrids_amd"))
import pamg  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 5
L = int(sys.argv[2]) if len(sys.argv) > 2 else 3
mesh = pamg.Mesh.read(os.path.join(ROOT, "tests", "meshes", "untitled8192.msh"))


def state(s):
    st = s.state()
    st["t_overlap"], st["t_overlap_old"] = s.overlap()
    return st


runs = {}
for sched in (1, 3):
    s = pamg.SemiImplicitIterative(mesh, S, L, n_smooth=4, solver=3, arith=1, fused=3)
    s.set_call_schedule(sched)
    s.run(3, 2)
    s.begin_timestep()
    s.vcycle(7)
    runs[sched] = state(s)
    s.close()
bad = [k for k in runs[1] if not np.array_equal(runs[1][k], runs[3][k])]
print("bitwise resident == per-cycle launches:", "yes" if not bad else f"NO {bad}", flush=True)

for sched in (1, 3):
    s = pamg.SemiImplicitIterative(mesh, S, L, n_smooth=4, solver=3, arith=1, fused=3)
    s.set_call_schedule(sched)
    fl = s.vcycle_flops()
    s.begin_timestep()
    s.vcycle(200)
    s.synchronize()
    for n in (200, 20):
        t0 = time.perf_counter()
        s.vcycle(n)
        s.synchronize()
        dt = time.perf_counter() - t0
        print(f"schedule {sched}: call of {n:3d} cycles {n / dt:9.1f} V-cycles/s  {dt / n * 1e3:.4f} ms/cycle  "
              f"{fl / (dt / n) / 1e12:.2f} TFLOP/s fp64", flush=True)
    s.run(5, 2)
    s.synchronize()
    t0 = time.perf_counter()
    s.run(50, 2)
    s.synchronize()
    dt = time.perf_counter() - t0
    print(f"schedule {sched}: time loop 50 x 2 {100 / dt:9.1f} V-cycles/s  {dt / 50 * 1e3:.4f} ms/step", flush=True)
    s.timing_enable(0x3F7F)
    s.timing_reset()
    s.vcycle(200)
    s.synchronize()
    t = s.timing()
    for k, v in t.items():
        if v["launches"]:
            print(f"   {k:16s} launches {v['launches']:4d} ms/launch {v['ms'] / v['launches']:.4f} "
                  f"GB/launch {v['bytes'] / v['launches'] / 1e9:.3f}", flush=True)
    s.close()
