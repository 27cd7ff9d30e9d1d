"""Edge cases of the hot path: a one-element mesh (tests/meshes/one_tri.msh -- every face a domain
boundary, one tile, a resident launch of one workgroup), calls of zero cycles or zero time steps, and the
largest n_split the resident call takes on it. Each GPU case is bitwise the oracle's restatement of the same
arithmetic (the oracle takes the device's source term s', as tests/test_contracted_oracle.py). The CPU case
pins the oracle on the one-element mesh against its own invariants (no reference output exists for this mesh:
parity on it is transitive through the oracle, which is pinned to the reference's goldens elsewhere)."""
import os

import numpy as np
import pytest

import goldens
import oracle_lib as O

MESH = "one_tri.msh"


def test_one_element_mesh_topology_and_oracle():
    """ReadMSH on one triangle: no neighbours (Neig 0 on every face, the domain boundary), and a V-cycle
    of the oracle reduces the level-1 residual of the step it starts."""
    m = O.read_msh(os.path.join(goldens.MESHES, MESH))
    assert m.U == 1
    np.testing.assert_array_equal(np.asarray(m.neig), 0)
    o = O.Oracle(m, 3, 3, ntime=1, n_multigrid=1)
    o.begin_timestep()
    o.get_residual(1)
    r0 = float(np.abs(o.get(O.RES, 1)).max())
    o.vcycle()
    o.get_residual(1)
    assert float(np.abs(o.get(O.RES, 1)).max()) < r0


def gpu_pair(S, L, arith=1, fused=3, ns=4, solver=3, op=0, cycle=0):
    import pamg
    path = os.path.join(goldens.MESHES, MESH)
    if op == 1:
        arith = 0   # (the face operator has one arithmetic)
    g = pamg.SemiImplicitIterative(pamg.Mesh.read(path), S, L, n_smooth=ns, solver=solver, fused=fused, arith=arith,
                                   op=op, cycle=cycle)
    o = O.Oracle(O.read_msh(path), S, L, n_smooth=ns, solver=solver, op=op, arith=arith)
    o.set_source(g.get(pamg.SOURCE, 1))
    return g, o


def assert_identical(g, o):
    sg, so = g.state(), o.state()
    for k in so:
        np.testing.assert_array_equal(sg[k], so[k], err_msg=k)
    for x, y in zip(g.overlap(), o.overlap()):
        np.testing.assert_array_equal(x, y)


@pytest.mark.gpu
@pytest.mark.parametrize("S,L,fused,arith", [
    (3, 3, 3, 1), (3, 3, 0, 0), (4, 4, 3, 0), (5, 3, 3, 1), (5, 3, 1, 1), (6, 3, 3, 1), (7, 4, 3, 0), (5, 5, 3, 1)])
def test_one_element_mesh_is_bitwise_the_oracle(S, L, fused, arith):
    """One un_ele: a resident call of ONE workgroup (n_split 5: k_vc_resb's single tile; 6-7: its quarter tiles),
    the per-step kernels (fused 0) and the pipelined call (fused 1), two time steps of three cycles."""
    g, o = gpu_pair(S, L, arith, fused)
    g.run(2, 3)
    for _ in range(2):
        o.begin_timestep()
        for _ in range(3):
            o.vcycle()
    assert_identical(g, o)
    g.close()


@pytest.mark.gpu
@pytest.mark.parametrize("cycle", [0, 1])
@pytest.mark.parametrize("S,L,ns", [(3, 3, 4), (5, 3, 4), (4, 2, 1)])
def test_one_element_face_operator_is_bitwise_the_oracle(S, L, ns, cycle):
    """The face operator where every face is a domain boundary: the halo snapshot holds only boundary words,
    the coarsest level's chain is one workgroup polling no neighbour."""
    g, o = gpu_pair(S, L, ns=ns, op=1, cycle=cycle)
    for s in (g, o):
        s.begin_timestep()
    g.vcycle(2)
    for _ in range(2):
        o.vcycle_corrected() if cycle else o.vcycle()
    assert_identical(g, o)
    g.close()


@pytest.mark.gpu
@pytest.mark.parametrize("op", [0, 1])
def test_zero_cycles_and_zero_steps_change_nothing(op):
    """pamg_vcycle(h, 0) and pamg_run(h, 0, n) are no-ops: the state after them is the state before, bit for
    bit, and a later call continues as if they had not been made."""
    import pamg
    m = pamg.Mesh.read(os.path.join(goldens.MESHES, "untitled8.msh"))
    a = pamg.SemiImplicitIterative(m, 3, 3, op=op)
    b = pamg.SemiImplicitIterative(m, 3, 3, op=op)
    for s in (a, b):
        s.begin_timestep()
        s.vcycle(1)
    before = a.state()
    a.vcycle(0)
    a.run(0, 2)
    after = a.state()
    for k in before:
        np.testing.assert_array_equal(after[k], before[k], err_msg=k)
    a.vcycle(2)
    b.vcycle(2)
    sa, sb = a.state(), b.state()
    for k in sa:
        np.testing.assert_array_equal(sa[k], sb[k], err_msg=k)
    a.close()
    b.close()


@pytest.mark.gpu
@pytest.mark.parametrize("mesh,own,n", [("one_tri.msh", [0], 2), ("untitled8.msh", [0, 0, 0, 0, 2, 2, 2, 2], 3)])
@pytest.mark.parametrize("op,cycle,fused", [(0, 0, 3), (0, 0, 0), (1, 0, 3), (1, 1, 3)])
def test_rank_owning_no_un_ele(mesh, own, n, op, cycle, fused):
    """A partition with a rank that owns nothing (more ranks than un_eles, or an owner map that skips a rank):
    that rank still takes part in every exchange and coarsest-level gather, with nothing to send, and the
    owning ranks' state equals the single domain's bit for bit (local-group transport)."""
    import pamg
    from pamg.solver import local_group, run_ranks
    m = pamg.Mesh.read(os.path.join(goldens.MESHES, mesh))
    owner = np.array(own, np.int32)
    full = pamg.SemiImplicitIterative(m, 3, 3, op=op, cycle=cycle, fused=fused)
    full.run(2, 2)
    ps = [pamg.SemiImplicitIterative(m, 3, 3, op=op, cycle=cycle, fused=fused, comm=(n, r, None, owner))
          for r in range(n)]
    local_group(ps)
    run_ranks(ps, lambda p: p.run(2, 2))
    ref, ref_ov = full.state(), full.overlap()
    for r, p in enumerate(ps):
        o = np.flatnonzero(owner == r)
        for k, v in p.state().items():
            np.testing.assert_array_equal(v, ref[k][:, :, o], err_msg=f"rank {r} {k}")
        for x, y in zip(p.overlap(), ref_ov):
            np.testing.assert_array_equal(x, y[:, :, o])
        p.close()
    full.close()
