"""Multi-rank halo path on CPU (gloo): the partitioned update_overlaps plan of
libpamg (pamg_plan_* host API -- the same plan the device pack / unpack kernels
and the RCCL send/recv segments follow) must reproduce the single-domain
reference halo.

Each rank owns an x-strip of untitled8192.msh. The rank's level fields are the
oracle's (pinned to the reference); packing, the per-peer exchange (ordered
like the grouped ncclSend/ncclRecv of pamg_api.cpp `halo`) and unpacking run
here with numpy + torch.distributed(gloo), and every rank's t_overlap /
t_overlap_old must equal the oracle's single-domain buffers on its elements.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import goldens
import oracle_lib as O
import pamg
from pamg.solver import HaloPlan

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

S, LEVELS = 3, 3


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def local_halo(rank, world, port, result_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        path = os.path.join(goldens.MESHES, "untitled8192.msh")
        mesh = pamg.Mesh.read(path)
        owner = mesh.x_strip_owner(world)
        o = O.Oracle(O.read_msh(path), S, LEVELS, ntime=1, n_multigrid=1)
        o.run()
        T, To = o.get(O.TNEW, 1), o.get(O.TOLD, 1)
        ref_ov, ref_ovo = o.overlap()
        plan = HaloPlan(mesh, S, 1, world, rank, owner)
        own = plan.owned
        assert np.array_equal(own, np.flatnonzero(owner == rank))
        nsub, slots, Ul = 4 ** S, 3 * 2 ** S, len(own)
        Tl = T[:, :, own].reshape(3, -1, order="F")      # (3, nsub*Ul): column s = q*nsub + sub
        Tol = To[:, :, own].reshape(3, -1, order="F")
        ov = np.zeros(slots * 3 * Ul)
        ovo = np.zeros(slots * 3 * Ul)
        for src, dst in zip(plan.local_src, plan.local_dst):
            ov[dst:dst + 3] = Tl[:, src]
            ovo[dst:dst + 3] = Tol[:, src]
        for i in range(len(plan.bc_val) // 2):
            for j in range(2):
                ov[plan.bc_dst[2 * i + j]] = plan.bc_val[2 * i + j]
                ovo[plan.bc_dst[2 * i + j]] = plan.bc_val[2 * i + j]
        send = np.zeros((len(plan.remote_src), 6))
        for e, src in enumerate(plan.remote_src):
            send[e, :3] = Tl[:, src]
            send[e, 3:] = Tol[:, src]
        reqs, recvs = [], []
        for q, peer in enumerate(plan.peers):
            a, b = plan.send_off[q], plan.send_off[q + 1]
            ra, rb = plan.recv_off[q], plan.recv_off[q + 1]
            buf = torch.zeros((rb - ra) * 6, dtype=torch.float64)
            recvs.append((ra, buf))
            reqs.append(dist.isend(torch.from_numpy(send[a:b].reshape(-1).copy()), int(peer)))
            reqs.append(dist.irecv(buf, int(peer)))
        for r in reqs:
            r.wait()
        for ra, buf in recvs:
            vals = buf.numpy().reshape(-1, 6)
            for e, dst in enumerate(plan.recv_dst[ra:ra + len(vals)]):
                ov[dst:dst + 3] = vals[e, :3]
                ovo[dst:dst + 3] = vals[e, 3:]
        ov = ov.reshape((slots, 3, Ul), order="F")
        ovo = ovo.reshape((slots, 3, Ul), order="F")
        ok = (np.array_equal(ov, ref_ov[:, :, own]) and np.array_equal(ovo, ref_ovo[:, :, own]))
        result_q.put((rank, ok, len(plan.remote_src), len(plan.recv_dst)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_partitioned_halo_exchange_matches_reference(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=local_halo, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
        assert p.exitcode == 0
    res = sorted(q.get(timeout=10) for _ in range(world))
    assert all(ok for _, ok, _, _ in res), res
    assert sum(n for _, _, n, _ in res) == sum(m for _, _, _, m in res) > 0


def test_single_rank_plan_has_no_remote_entries():
    mesh = pamg.Mesh.read(os.path.join(goldens.MESHES, "untitled8.msh"))
    p = HaloPlan(mesh, 3, 1, 1, 0, None)
    assert len(p.remote_src) == 0 and len(p.recv_dst) == 0 and len(p.peers) == 0
    assert len(p.owned) == mesh.U


def test_bench_rank_that_never_joins_ends_the_run_with_an_error_line():
    """`bench.py --gpus 2` whose rank 1 never starts. RCCL's initialisation cannot be bounded
    (profiles/r06_rccl_init_probe.txt), so bench.py meets every rank in a gloo rendezvous with a timeout before
    pamg_comm_init: rank 0 must exit non-zero within the bound, with one JSON line naming its rank and the error,
    instead of hanging. (Runs on the CPU: the rendezvous fails before any GPU work.)"""
    import json
    import socket
    import subprocess
    import sys
    import time
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    env = dict(os.environ, RANK="0", LOCAL_RANK="0", WORLD_SIZE="2", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
               PAMG_BENCH_RENDEZVOUS_S="10")
    t0 = time.time()
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1"],
                       env=env, capture_output=True, text=True, timeout=240)
    dt = time.time() - t0
    assert r.returncode != 0, r.stdout
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout + r.stderr
    d = json.loads(lines[0])
    assert d["value"] is None and d["rank"] == 0 and d["world_size"] == 2 and d["error"], d
    assert dt < 200, dt
