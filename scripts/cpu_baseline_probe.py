"""Check of bench.py's cpu_baseline scaling: the reference's own fp64 build (1 core) at
n_split = 5 on the 512-element strip bench.py samples and on the full untitled8192.msh, plus
untitled8192 at n_split = 3 and 4 (the per-sub-element cost across sizes). Every number is the
reference's own `cpu_time for time_loop` window. ~5 min of CPU on the GPU box's host; writes a table to stdout
(committed as archive/profiles/r02_cpu_baseline_probe.txt)."""
import os
import sys
import tempfile

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "p-a_multigrids_amd"))
import bench  # noqa: E402
import pamg  # noqa: E402

print(f"host: {bench.host_cpu()}, 1 core (taskset -c 0), reference fp64 build (oracle/_ref/pamg_ref_fp64)")
with tempfile.TemporaryDirectory() as d:
    strip = os.path.join(d, "strip.msh")
    pamg.Mesh.strip(*bench.CPU_STRIP).write_msh(strip)
    full = bench.MESH
    rows = []
    for name, path, U, S, nt, nmg in (("strip 32x8x2", strip, 512, 5, 1, 1), ("strip 32x8x2", strip, 512, 5, 1, 2),
                                      ("untitled8192", full, 8192, 3, 1, 1), ("untitled8192", full, 8192, 5, 1, 1)):
        t = bench.run_reference(path, S, nt, nmg, timeout=1500)
        nsub = U * 4 ** S
        per = None if t is None else t / nmg
        rows.append((name, U, S, nmg, t, per, None if t is None else per / nsub * 1e9))
        print(f"{name:>14} U={U:<5} n_split={S} ntime={nt} n_multigrid={nmg}: time_loop {t:.2f} s, "
              f"{per:.2f} s per V-cycle, {per / nsub * 1e9:.1f} ns per level-1 sub-element per V-cycle", flush=True)
    s5 = [r for r in rows if r[0] == "strip 32x8x2" and r[3] == 1][0]
    f5 = [r for r in rows if r[0] == "untitled8192" and r[2] == 5][0]
    print(f"untitled8192 / strip at n_split=5 (1 V-cycle): {f5[4] / s5[4]:.2f}x for {8192 // 512}x the elements")
