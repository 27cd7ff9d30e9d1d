"""The north star's HBM roofline kernel (k_sweep_assembled, 168 B per sub-element) and the matrix-free sweep
beside it, on bench.py's level 1 (untitled8192, n_split 5): average of `--launches` evented launches after a
warm-up, repeated `--reps` times (GPU box only). The block layout comes from PAMG_ASM_LAYOUT, the plane gap
from PAMG_PITCH_PAD (archive/scripts/r5_e.sh runs the variants in separate processes)."""
import argparse
import os
import sys

import torch  # noqa: F401

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "p-a_multigrids_amd"))
import pamg  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--launches", type=int, default=60)
ap.add_argument("--reps", type=int, default=3)
a = ap.parse_args()
s = pamg.SemiImplicitIterative(pamg.Mesh.read(os.path.join(ROOT, "tests", "meshes", "untitled8192.msh")), 5, 3)
s.begin_timestep()
s.sweep_bench(10, True)
s.sweep_bench(10, False)
tag = f"layout={os.environ.get('PAMG_ASM_LAYOUT', 'default')} pad={os.environ.get('PAMG_PITCH_PAD', '0')}"
for r in range(a.reps):
    ma, ba = s.sweep_bench(a.launches, True)
    ms, bs = s.sweep_bench(a.launches, False)
    print(f"{tag}: assembled {ma:.4f} ms {ba / ma / 1e6:.1f} GB/s frac {ba / ma / 1e6 / 8000:.3f} | "
          f"stencil {ms:.4f} ms frac {bs / ms / 1e6 / 8000:.3f}", flush=True)
s.close()
