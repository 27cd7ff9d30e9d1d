"""Mesh ingest time (host, 1 core): pamg_msh_read (O(U) edge hash) and the binary mesh cache
against the reference's ReadMSH + O(U^2) CheckNeig (the oracle's literal restatement,
oracle/pamg_oracle.c, pinned to the reference; Msh2Tri.F90:323-330, 776-963 -- 99 % of a large
run in grofiling.txt:6-8). Synthetic strips written as gmsh 2.2 (pamg_msh_write).
Writes a table to stdout; the committed copy is archive/profiles/r02_ingest_timing.txt."""
import os
import sys
import tempfile
import time

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "p-a_multigrids_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402

import oracle_lib as O  # noqa: E402
import pamg  # noqa: E402

ORACLE_MAX_U = int(os.environ.get("ORACLE_MAX_U", "32768"))
print(f"host: {open('/proc/cpuinfo').read().split('model name')[1].split(':')[1].splitlines()[0].strip()}")
print(f"{'U':>9} {'msh MB':>7} {'pamg_msh_read s':>16} {'cache write s':>14} {'cache read s':>13} "
      f"{'reference CheckNeig s':>22}")
with tempfile.TemporaryDirectory() as d:
    for nx, ny in ((64, 16), (128, 32), (256, 64), (512, 128), (1024, 256), (2048, 512)):
        U = 2 * nx * ny
        path = os.path.join(d, f"s{U}.msh")
        pamg.Mesh.strip(nx, ny).write_msh(path)
        t0 = time.perf_counter()
        m = pamg.Mesh.read(path)
        t_read = time.perf_counter() - t0
        cache = path + ".cache"
        t0 = time.perf_counter()
        m.save(cache)
        t_save = time.perf_counter() - t0
        t0 = time.perf_counter()
        c = pamg.Mesh.load(cache)
        t_load = time.perf_counter() - t0
        assert np.array_equal(c.neig, m.neig) and np.array_equal(c.X, m.X)
        t_ref = ""
        if U <= ORACLE_MAX_U:
            t0 = time.perf_counter()
            o = O.read_msh(path)
            t_ref = f"{time.perf_counter() - t0:.3f}"
            assert np.array_equal(o.neig, m.neig) and np.array_equal(o.dir, m.dir)
        print(f"{U:>9} {os.path.getsize(path) / 1e6:>7.1f} {t_read:>16.3f} {t_save:>14.4f} {t_load:>13.4f} "
              f"{t_ref:>22}", flush=True)
