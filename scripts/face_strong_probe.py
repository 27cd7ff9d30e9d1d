"""The face-coupled operator (op = 1) on partitions: per-rank V-cycle time of the x-strip partition of
untitled8192 at N = 1, 2, 4, 8 ranks, simulated on one GPU (rank 0's partition, detached: the halo
refresh and the sweeps of every rank run, the exchange itself does not -- its latency is the RCCL
transport's, a multi-GPU node's), beside the single domain's fused cycle. On a partition every sweep of
levels 1-3 is the halo refresh, the exchange and one tile launch (pamg_api.cpp smooth, op = 1): no chain
and no two-sweep passes, which need the neighbours' words inside the launch.
Usage: python scripts/face_strong_probe.py [n_split] [cycles]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "p-a_multigrids_amd"))
import pamg  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 5
K = int(sys.argv[2]) if len(sys.argv) > 2 else 10
mesh = pamg.Mesh.read(os.path.join(ROOT, "tests", "meshes", "untitled8192.msh"))
base = None
for n in (1, 2, 4, 8):
    comm = None if n == 1 else (n, 0, None, mesh.x_strip_owner(n))
    s = pamg.SemiImplicitIterative(mesh, S, 3, n_smooth=4, solver=3, op=1, comm=comm)
    s.begin_timestep()
    s.vcycle(3)
    s.synchronize()
    t0 = time.perf_counter()
    s.vcycle(K)
    s.synchronize()
    dt = (time.perf_counter() - t0) / K * 1e3
    s.timing_enable(0x7F7F)
    s.timing_stride(1)
    s.timing_reset()
    s.vcycle(K)
    s.synchronize()
    tm = s.timing()
    if base is None:
        base = dt
    kinds = {k: (v["launches"] // K, round(v["ms"] / K, 4)) for k, v in tm.items() if v["launches"]}
    print(f"op=1 S={S} N={n} (rank 0: {s.U} un_eles, {'fused single domain' if n == 1 else 'partition, detached'}): "
          f"{dt:.4f} ms/cycle ({1e3 / dt:.1f} V-cycles/s per rank; N=1 / N = {base / dt:.2f}x); per cycle "
          f"(launches, ms): {kinds}", flush=True)
    s.close()
