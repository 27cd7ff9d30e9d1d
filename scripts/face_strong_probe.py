"""The face-coupled operator (op = 1) on partitions: per-rank V-cycle time of the x-strip partition of
untitled8192 at N = 1, 2, 4, 8 ranks, simulated on one GPU (rank 0's partition, detached: the halo
refresh and the sweeps of every rank run, the exchange itself does not -- its latency is the RCCL
transport's, a multi-GPU node's), beside the single domain's fused cycle. On a partition every sweep of
levels 1-2 is the halo refresh, the exchange and one tile launch (pamg_api.cpp smooth, op = 1): no
two-sweep passes, which need the neighbours' iterate inside the launch. Level 3 is agglomerated (round 6):
each cycle gathers the ranks' level-3 RHS into a replica of the whole level and every rank runs the
single-domain chain on it; a detached rank copies only its own block, so the gather's cross-GPU part is
charged as a model: the bytes each rank receives ((N-1)/N of the level's 3-plane RHS, 12.6 MB at n_split 5)
over the N-1 xGMI links at XGMI_GBS each in parallel, plus XGMI_LAT_US per gather.
Usage: python scripts/face_strong_probe.py [n_split] [cycles] [agg 0|1]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "p-a_multigrids_amd"))
import pamg  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 5
K = int(sys.argv[2]) if len(sys.argv) > 2 else 10
if len(sys.argv) > 3:
    os.environ["PAMG_FACE_AGG"] = sys.argv[3]
AGG = os.environ.get("PAMG_FACE_AGG", "1") != "0"
XGMI_GBS, XGMI_LAT_US = 48.0, 15.0   # per link and direction, achieved by a 1.6 MB RCCL p2p transfer (assumed)
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
    s.timing_enable(0x27F7F)
    s.timing_stride(1)
    s.timing_reset()
    s.vcycle(K)
    s.synchronize()
    tm = s.timing()
    if base is None:
        base = dt
    kinds = {k: (v["launches"] // K, round(v["ms"] / K, 4)) for k, v in tm.items() if v["launches"]}
    charge = 0.0
    if n > 1 and AGG:
        lvl3 = 3 * 8 * mesh.U * 4 ** (S - 2)   # the level-3 RHS of the whole mesh (3 planes, fp64)
        per_link = lvl3 / n                    # each peer's block arrives over its own link
        gathers = tm["coarse_gather"]["issued"] / K   # per cycle (the RHS; tnew once per call)
        charge = gathers * (per_link / (XGMI_GBS * 1e9) * 1e3 + XGMI_LAT_US * 1e-3)
    dtc = dt + charge
    print(f"op=1 S={S} N={n} agg={int(AGG)} (rank 0: {s.U} un_eles, {'fused single domain' if n == 1 else 'partition, detached'}): "
          f"{dt:.4f} ms/cycle measured, {dtc:.4f} with the modeled cross-GPU gather ({charge * 1e3:.1f} us) "
          f"({1e3 / dtc:.1f} V-cycles/s per rank; N=1 / N = {base / dtc:.2f}x); per cycle "
          f"(launches, ms): {kinds}", flush=True)
    s.close()
