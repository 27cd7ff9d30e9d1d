"""The face-coupled operator (op = 1) on bench.py's mesh: V-cycles/s of the reference's cycle
and of the corrected cycle, and the per-kernel-class times and algorithmic bytes.
Usage: python scripts/face_probe.py [n_split]"""
import os
import sys
import time

if os.environ.get("PAMG_PROBE_TORCH", "1") != "0":
    import torch  # noqa: F401  (as bench.py: the HIP runtime comes up through torch)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "p-a_multigrids_amd"))
import pamg  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 5
CYCLES = [int(c) for c in sys.argv[2].split(",")] if len(sys.argv) > 2 else [0, 1]
mesh = pamg.Mesh.read(os.path.join(ROOT, "tests", "meshes", "untitled8192.msh"))
for cycle in CYCLES:
    s = pamg.SemiImplicitIterative(mesh, S, 3, n_smooth=4, solver=3, op=1, cycle=cycle)
    s.begin_timestep()
    s.vcycle(3)
    s.synchronize()
    n = 10
    t0 = time.perf_counter()
    s.vcycle(n)
    s.synchronize()
    dt = (time.perf_counter() - t0) / n
    s.timing_enable(0x7F7F)
    s.timing_stride(1)
    s.timing_reset()
    s.vcycle(n)
    s.synchronize()
    tm = s.timing()
    print(f"op=1 cycle={cycle} S={S}: {1 / dt:.1f} V-cycles/s ({dt * 1e3:.3f} ms per cycle)", flush=True)
    for k, v in tm.items():
        if v["launches"]:
            ms = v["ms"] / n
            print(f"   {k:14s} {v['launches'] // n:4d} launches/cycle {ms:.4f} ms/cycle "
                  f"{v['bytes'] / (v['ms'] * 1e-3) / 1e9 if v['ms'] else 0:.0f} GB/s (algorithmic)", flush=True)
    s.close()
# PAMG_PROBE_MAPS=<path>: the process's mappings at the end (resolves the PCs of a crash at exit)
if os.environ.get("PAMG_PROBE_MAPS"):
    with open("/proc/self/maps") as f, open(os.environ["PAMG_PROBE_MAPS"], "w") as o:
        o.write(f.read())
