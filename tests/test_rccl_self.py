"""The RCCL transport itself on one GPU: a one-rank communicator with a self-peer halo plan.

RCCL refuses two ranks on one GPU, so the multi-rank tests (tests/test_multirank.py) run the
exchange path through the device-copy transport. Here the halo words across the parts of a
virtual partition are the plan's "remote" words with this rank as their peer
(pamg_comm_init_self): the V-cycle launches pack them into the send buffers, `exchange()`
issues the grouped ncclSend / ncclRecv (ncclGroupStart/End, splitting.F90:1210-1397's words)
on the one-rank communicator, the unpack kernel writes them into t_overlap, and the async
error state is polled (ncclCommGetAsyncError) at the end of every call. Every field of every
level, t_overlap and t_overlap_old must equal the plain single domain's bit for bit.
"""
import os

import numpy as np
import pytest

import goldens
import pamg

pytestmark = pytest.mark.gpu


def _pair(mesh, S, L, parts, **kw):
    full = pamg.SemiImplicitIterative(mesh, S, L, **kw)
    part = mesh.x_strip_owner(parts)
    s = pamg.SemiImplicitIterative(mesh, S, L, self_peer=(pamg.unique_id(), part), **kw)
    assert s.comm_info()[0] == "rccl"
    return full, s


def _same(full, s):
    a, b = full.state(), s.state()
    for k in a:
        np.testing.assert_array_equal(b[k], a[k], err_msg=k)
    for x, y in zip(s.overlap(), full.overlap()):
        np.testing.assert_array_equal(x, y)


@pytest.mark.parametrize("how", ["vcycle", "run", "per_step", "halo_every_cycle"])
def test_rccl_self_peer_exchange_is_the_single_domain(how):
    mesh = pamg.Mesh.read(os.path.join(goldens.MESHES, "untitled8192.msh"))
    kw = dict(n_smooth=4, solver=3, arith=1)
    if how == "per_step":
        kw["fused"] = 0            # an exchange after every smoother call
    if how == "halo_every_cycle":
        kw["halo_exchange"] = 1    # an exchange after every cycle, on the comm stream
    full, s = _pair(mesh, 3, 3, 4, **kw)
    for x in (full, s):
        if how == "run":
            x.run(3, 2)
        else:
            x.begin_timestep()
            x.vcycle(3)
    _same(full, s)
    s.close()
    full.close()


def test_rccl_self_peer_face_operator():
    """op = 1 reads the halo every sweep: the words exchanged through RCCL are load-bearing"""
    mesh = pamg.Mesh.read(os.path.join(goldens.MESHES, "irregular.msh"))
    full, s = _pair(mesh, 3, 3, 3, op=1, cycle=1, n_smooth=2)
    s.timing_enable(1 << 17)   # PAMG_K_COARSE_GATHER
    s.timing_reset()
    for x in (full, s):
        x.begin_timestep()
        x.vcycle(2)
    _same(full, s)
    # the coarsest level agglomerated: its RHS crosses RCCL (to this rank itself) once per cycle
    assert s.timing()["coarse_gather"]["issued"] == 2, s.timing()["coarse_gather"]


def test_rccl_self_peer_face_operator_reference_cycle():
    """the reference cycle on the face operator through RCCL: the coarsest level's tnew gathered once per call,
    its RHS once per cycle (the bench's op = 1 configuration, n_split 5)"""
    mesh = pamg.Mesh.read(os.path.join(goldens.MESHES, "untitled8192.msh"))
    full, s = _pair(mesh, 5, 3, 4, op=1, cycle=0, n_smooth=4)
    s.timing_enable(1 << 1 | 1 << 17)   # PAMG_K_SMOOTH (levels >= 2), PAMG_K_COARSE_GATHER
    s.timing_reset()
    for x in (full, s):
        x.begin_timestep()
        x.vcycle(3)
        x.vcycle(2)
    _same(full, s)
    tm = s.timing()
    assert tm["coarse_gather"]["issued"] == 5 + 2, tm["coarse_gather"]
    # level 2 one launch per executed sweep (2 (n_smooth - 1) a cycle, + 1 in a call's last), the coarsest level as
    # the replica's chain: one launch a cycle, two in a call's last -- not 62 launches and exchanges a cycle
    assert tm["smooth"]["issued"] <= 5 * (2 * 3 + 1) + 2 * 2, tm["smooth"]


def test_rccl_self_peer_early_exchange_is_hidden():
    """The resident call's per-call exchange starts on the device signal raised when the tiles with remote
    faces (scheduled first) have finished, and runs through RCCL while the other tiles compute: one early
    exchange per call, the state bitwise the single domain's, and the exchange (ncclSend / ncclRecv and the
    unpack) ends before the resident launch does. The shape of one rank of config 4 on 8 GPUs: 1,024 un_eles
    at n_split 5 (a 32 x 16 x 2 strip, 1.33 rounds of resident workgroups), one cut of 16 faces' rows; on the
    full mesh's 10.7 full rounds the exchange's kernels only find free CUs in the launch's tail."""
    mesh = pamg.Mesh.strip(32, 16)
    full, s = _pair(mesh, 5, 3, 2, n_smooth=4, solver=3, arith=1)
    for x in (full, s):
        x.begin_timestep()
        x.vcycle(5)
    s.timing_enable(0xFFFF)
    s.timing_reset()
    for x in (full, s):
        x.vcycle(20)
    _same(full, s)
    tm = s.timing()
    assert tm["vcycle_res"]["issued"] == 1 and tm["halo_early"]["issued"] == 1, tm
    t0, t1, t2 = s.early_exchange_times()
    print(f"early exchange: start {t0:.1f} us, end {t1:.1f} us, launch end {t2:.1f} us")
    assert 0 <= t0 <= t1 < t2, (t0, t1, t2)
    s.close()
    full.close()


def test_timing_read_right_after_an_early_exchange():
    """the early exchange's spans sit on the comm stream and the call returns without joining it.
    On the full bench mesh the exchange can outlast the launch (it only finds free CUs in the launch's tail), so
    timing() read straight after the call -- no state() or overlap() first, which would settle -- must still
    wait for those spans instead of failing on an event that has not completed."""
    mesh = pamg.Mesh.read(os.path.join(goldens.MESHES, "untitled8192.msh"))
    part = mesh.x_strip_owner(8)
    s = pamg.SemiImplicitIterative(mesh, 5, 3, n_smooth=4, solver=3, arith=1, self_peer=(pamg.unique_id(), part))
    s.begin_timestep()
    s.timing_enable(0xFFFF)
    s.timing_reset()
    for _ in range(3):
        s.vcycle(1)
        tm = s.timing()
    assert tm["halo_early"]["issued"] == 3 and tm["halo_early"]["launches"] == 3, tm["halo_early"]
    assert tm["halo_early"]["ms"] > 0
    s.close()

