"""Partitioned runs through the real multi-rank exchange path on one GPU.

`pamg_comm_local_group` binds n partition handles of one process into a transport whose
halo exchange is the RCCL path itself -- the level-1 words packed by the V-cycle launches
into alternating send buffers, the exchange on the comm stream overlapped with the next
cycle (`halo_async`), the buffer reuse guarded by the send-completion events, `join_comm`
at the end of the call -- with ncclSend / ncclRecv replaced by device-to-device copies
between the handles. Each partition runs in its own host thread, as one process per rank
does, and ranks meet at every exchange. Only the RCCL transport itself is left for a
multi-GPU node (RCCL refuses two ranks on one GPU).

Every partitioned state -- all fields of all levels on the rank's un_eles, t_overlap and
t_overlap_old -- must equal the single-domain run's bit for bit (the exchange is a copy).
"""
import os

import numpy as np
import pytest

import goldens
import pamg
from pamg.solver import local_group, run_ranks

pytestmark = pytest.mark.gpu


def owners(mesh, kind, n):
    return mesh.x_strip_owner(n) if kind == "strip" else mesh.block_owner(n)


def drive(s, how):
    if how == "run":
        s.run(3, 2)
    elif how == "vcycle20":
        s.begin_timestep()
        s.vcycle(20)
    elif how == "calls":   # public per-step and fused calls mixed
        s.begin_timestep()
        s.vcycle(2)
        s.begin_timestep()
        s.vcycle(1)
        s.vcycle(3)
    else:
        raise ValueError(how)


def check_parts(full, parts, owner):
    ref_state = full.state()
    ref_ov = full.overlap()
    for r, p in enumerate(parts):
        own = np.flatnonzero(owner == r)
        assert p.U == len(own)
        for k, v in p.state().items():
            np.testing.assert_array_equal(v, ref_state[k][:, :, own], err_msg=f"rank {r} {k}")
        for x, y in zip(p.overlap(), ref_ov):
            np.testing.assert_array_equal(x, y[:, :, own], err_msg=f"rank {r} t_overlap")


CASES = [
    # mesh, n_split, levels, parts, owner, fused, halo_exchange, drive, call schedule
    ("untitled8192.msh", 5, 3, 8, "strip", 3, 1, "vcycle20", 0),   # config 4, exchange after every cycle
    ("untitled8192.msh", 5, 3, 8, "strip", 3, 1, "run", 0),
    ("untitled8192.msh", 5, 3, 8, "strip", 3, 0, "run", 0),
    ("untitled8192.msh", 5, 3, 8, "strip", 3, 0, "run", 1),        # the RHSF launch on a partition
    ("untitled8192.msh", 3, 3, 4, "block", 3, 1, "calls", 2),
    ("untitled8192.msh", 3, 3, 4, "block", 0, 0, "run", 0),        # per-step kernels: exchange per smoother call
    ("irregular.msh", 6, 3, 8, "strip", 3, 0, "run", 0),           # config 5: 11 un_eles on 8 ranks
    ("irregular.msh", 6, 3, 8, "block", 3, 1, "vcycle20", 0),
    ("irregular.msh", 6, 3, 8, "strip", 1, 1, "calls", 0),
    ("900_ele.msh", 3, 2, 3, "block", 3, 1, "run", 1),
]


@pytest.mark.parametrize("mesh,S,L,nparts,kind,fused,exch,how,sched", CASES)
def test_local_group_matches_single_domain(mesh, S, L, nparts, kind, fused, exch, how, sched):
    m = pamg.Mesh.read(os.path.join(goldens.MESHES, mesh))
    full = pamg.SemiImplicitIterative(m, S, L, fused=0, arith=1)
    drive(full, how)
    owner = owners(m, kind, nparts)
    parts = [pamg.SemiImplicitIterative(m, S, L, comm=(nparts, r, None, owner), fused=fused, arith=1,
                                        halo_exchange=exch) for r in range(nparts)]
    local_group(parts)
    assert all(p.comm_info()[0] == "local" for p in parts)
    for p in parts:
        if sched:
            p.set_call_schedule(sched)
        p.timing_enable(1 << 6)   # count the exchanges (PAMG_K_HALO)
        p.timing_reset()
    run_ranks(parts, lambda p: drive(p, how))
    check_parts(full, parts, owner)
    assert all(p.timing()["halo"]["issued"] > 0 for p in parts)
    for p in parts:
        p.close()


@pytest.mark.parametrize("S,L,kind,nparts,solver", [(5, 3, "strip", 8, 3), (3, 3, "block", 4, 3), (4, 2, "strip", 2, 2)])
def test_local_group_exchange_every_cycle_inside_the_resident_call(S, L, kind, nparts, solver):
    """halo_exchange = 1 keeps the resident call (k_vc_resb / k_vc_res with XC): every cycle but
    the last packs its remote words into the ring and publishes the cycle on the device signal; the
    comm stream waits on it and exchanges that cycle's words while the launch runs on. One launch,
    one exchange per cycle, and the state is the single domain's bit for bit."""
    m = pamg.Mesh.read(os.path.join(goldens.MESHES, "untitled8192.msh"))
    kw = dict(solver=solver, arith=1)
    full = pamg.SemiImplicitIterative(m, S, L, fused=0, **kw)
    drive(full, "vcycle20")
    owner = owners(m, kind, nparts)
    parts = [pamg.SemiImplicitIterative(m, S, L, comm=(nparts, r, None, owner), fused=3, halo_exchange=1, **kw)
             for r in range(nparts)]
    local_group(parts)
    for p in parts:
        p.timing_enable(0x7F7F)
        p.timing_reset()
    run_ranks(parts, lambda p: drive(p, "vcycle20"))
    check_parts(full, parts, owner)
    for p in parts:
        tm = p.timing()
        assert tm["vcycle_res"]["issued"] == 1, tm["vcycle_res"]
        assert tm["halo"]["issued"] == 20, tm["halo"]
        p.close()


@pytest.mark.parametrize("S,L,kind,nparts,solver", [(5, 3, "strip", 8, 3), (3, 3, "block", 4, 1), (6, 3, "strip", 8, 3)])
def test_local_group_corrected_resident_call(S, L, kind, nparts, solver):
    """The corrected cycle's resident call (k_vc_corr) on partitions: the level-1 halo words of the
    call's last smoother call packed by the launch and exchanged once after it; every field and both
    halo arrays of every rank equal the single domain's per-step sequence, bit for bit."""
    mesh = "irregular.msh" if S == 6 else "untitled8192.msh"
    m = pamg.Mesh.read(os.path.join(goldens.MESHES, mesh))
    kw = dict(solver=solver, arith=1, cycle=1)
    full = pamg.SemiImplicitIterative(m, S, L, fused=0, **kw)
    drive(full, "calls")
    owner = owners(m, kind, nparts)
    parts = [pamg.SemiImplicitIterative(m, S, L, comm=(nparts, r, None, owner), fused=3, **kw) for r in range(nparts)]
    local_group(parts)
    for p in parts:
        p.timing_enable(0x7F7F)
        p.timing_reset()
    run_ranks(parts, lambda p: drive(p, "calls"))
    check_parts(full, parts, owner)
    for p in parts:
        tm = p.timing()
        if p.U:
            assert tm["vcycle_corr"]["issued"] == 3, tm["vcycle_corr"]
        p.close()


def test_local_group_halo_mode_per_sweep():
    """halo_mode = 1 with the per-step kernels: one launch per sweep and an exchange after every
    sweep (the reference's halo schedule, :555), on 2 ranks."""
    m = pamg.Mesh.read(os.path.join(goldens.MESHES, "untitled8192.msh"))
    full = pamg.SemiImplicitIterative(m, 3, 3, fused=0)
    full.run(2, 2)
    owner = m.x_strip_owner(2)
    parts = [pamg.SemiImplicitIterative(m, 3, 3, comm=(2, r, None, owner), halo_mode=1, fused=0) for r in range(2)]
    local_group(parts)
    run_ranks(parts, lambda p: p.run(2, 2))
    check_parts(full, parts, owner)


def test_local_group_reports_a_missing_peer(monkeypatch):
    """A rank whose peer never reaches the exchange fails with PAMG_ERR_COMM after
    PAMG_COMM_TIMEOUT_S instead of hanging."""
    monkeypatch.setenv("PAMG_COMM_TIMEOUT_S", "2")
    m = pamg.Mesh.read(os.path.join(goldens.MESHES, "untitled8.msh"))
    owner = m.block_owner(2)
    parts = [pamg.SemiImplicitIterative(m, 2, 2, comm=(2, r, None, owner)) for r in range(2)]
    local_group(parts)
    with pytest.raises(pamg.PamgError) as e:
        parts[0].run(1, 1)
    assert e.value.rc == -5 and "timed out" in str(e.value)


def test_comm_info_names_the_rccl_library():
    m = pamg.Mesh.read(os.path.join(goldens.MESHES, "untitled8.msh"))
    s = pamg.SemiImplicitIterative(m, 2, 2)
    kind, version, path = s.comm_info()
    assert kind == "none" and version >= 20000 and "rccl" in os.path.basename(path)


XE_CASES = [
    # mesh, n_split, levels, parts, owner, drive
    ("untitled8192.msh", 5, 3, 8, "strip", "vcycle20"),   # config 4's shape: k_vc_resb
    ("untitled8192.msh", 5, 3, 8, "block", "calls"),
    ("untitled8192.msh", 3, 3, 4, "block", "calls"),      # k_vc_res (16 un_eles per tile)
    ("irregular.msh", 6, 3, 8, "strip", "vcycle20"),      # config 5: tiles are quarters of an un_ele
]


@pytest.mark.parametrize("mesh,S,L,nparts,kind,how", XE_CASES)
def test_local_group_early_per_call_exchange(mesh, S, L, nparts, kind, how):
    """halo_exchange = 0 on a partition: the resident call's per-call exchange starts early -- the tiles
    holding a remote face run first (the launch's tile order), count their ends once their send words are
    written through, and the last raises the device signal on which the comm stream starts the exchange
    while the other tiles run (pamg_api.cpp vcycle_fused). One early exchange per
    vcycle call; the state is the single domain's bit for bit."""
    m = pamg.Mesh.read(os.path.join(goldens.MESHES, mesh))
    full = pamg.SemiImplicitIterative(m, S, L, fused=0, arith=1)
    drive(full, how)
    owner = owners(m, kind, nparts)
    parts = [pamg.SemiImplicitIterative(m, S, L, comm=(nparts, r, None, owner), fused=3, arith=1, halo_exchange=0)
             for r in range(nparts)]
    local_group(parts)
    for p in parts:
        p.timing_enable(0xFFFF)
        p.timing_reset()
    run_ranks(parts, lambda p: drive(p, how))
    check_parts(full, parts, owner)
    calls = 1 if how == "vcycle20" else 3
    for p in parts:
        tm = p.timing()
        assert tm["vcycle_res"]["issued"] == calls, tm["vcycle_res"]
        assert tm["halo_early"]["issued"] == calls, tm["halo_early"]
        t = p.early_exchange_times()
        assert t is not None and 0 <= t[0] <= t[1] and t[2] > 0, t
        p.close()
