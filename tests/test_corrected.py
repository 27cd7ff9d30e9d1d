"""The corrected V-cycle (pamg_params.cycle = 1).

The reference's cycle (A3) discards its coarse correction, restricts the previous
cycle's residual and has the A x - b sign; the corrected cycle keeps the reference's
levels, operators, smoother, restrictor weights and the P1 interpolation its
prolongator encodes, and fixes those defects (oracle/pamg_oracle.c
orc_vcycle_corrected). No reference output exists for it: the HIP path is pinned to
the oracle restatement, whose every building block (smoother, residual products,
restrictor, geometry) is pinned to the reference (tests/test_oracle_golden.py).
Tolerance (check_corrected): every field's error is measured against the level-1 field of
its kind (tnew-like against max|tnew_L1|, RHS / residual against max|RHS_L1|, the halo
against its own max), at 1e-12. Level 1 is then held to 1e-12 relative; the coarse levels
hold corrections and restricted residuals whose own magnitudes can be 1e-9 of the level-1
terms they were computed from (the restrictor's means cancel), so what matters -- and what
fp64 determines -- is their absolute accuracy on the solution's scale. The only operation
that differs between the two paths is the device sine of the level-1 source term.
"""
import os

import numpy as np
import pytest

import goldens
import oracle_lib as O

def check_corrected(sg, so, tol=1e-12):
    scale = {"t": float(np.abs(so["tnew_L1"]).max()), "r": float(np.abs(so["RHS_L1"]).max())}
    for k, v in so.items():
        if k.startswith("t_overlap"):
            sc = max(float(np.abs(v).max()), 1e-300)
        else:
            sc = scale["t"] if k.startswith(("tnew", "told")) else scale["r"]
        e = float(np.abs(np.asarray(sg[k]) - v).max()) / sc
        assert e <= tol, (k, e)


CASES = [("untitled8.msh", 3, 3), ("irregular.msh", 3, 3), ("900_ele.msh", 2, 2), ("untitled8192.msh", 3, 3),
         ("untitled8.msh", 2, 1)]


def oracle_run(mesh, S, L, cycles, coarse_solver=0):
    om = O.read_msh(os.path.join(goldens.MESHES, mesh))
    o = O.Oracle(om, S, L, ntime=1, n_multigrid=cycles, coarse_solver=coarse_solver)
    o.begin_timestep()
    norms = []
    for _ in range(cycles):
        o.vcycle_corrected()
        norms.append(float(np.linalg.norm(o.get(O.RES, 1))))
    return o, norms


@pytest.mark.parametrize("mesh,S,L", [("untitled8.msh", 3, 3), ("900_ele.msh", 2, 2), ("irregular.msh", 3, 3)])
def test_oracle_corrected_cycle_converges_faster(mesh, S, L):
    """CPU: the fine residual b - A x shrinks cycle by cycle, and after 6 cycles it is below a
    fifth of the residual the reference's cycle reports (its coarse correction is dead and its
    legs restart one sweep back)."""
    _, norms = oracle_run(mesh, S, L, 6)
    assert all(b < a for a, b in zip(norms, norms[1:])), norms
    om = O.read_msh(os.path.join(goldens.MESHES, mesh))
    o = O.Oracle(om, S, L, ntime=1, n_multigrid=1)
    o.begin_timestep()
    for _ in range(6):
        o.vcycle()
    faithful = float(np.linalg.norm(o.get(O.RES, 1)))
    assert norms[-1] < 0.2 * faithful, (norms[-1], faithful)


@pytest.mark.gpu
@pytest.mark.parametrize("mesh,S,L", CASES)
@pytest.mark.parametrize("coarse_solver", [0, 1])
def test_corrected_cycle_matches_oracle(mesh, S, L, coarse_solver):
    import pamg
    if L == 1 and coarse_solver == 1:
        pytest.skip("one level: nothing coarse to solve")
    cycles = 3
    o, norms = oracle_run(mesh, S, L, cycles, coarse_solver)
    s = pamg.SemiImplicitIterative(pamg.Mesh.read(os.path.join(goldens.MESHES, mesh)), S, L, cycle=1,
                                   coarse_solver=coarse_solver)
    s.begin_timestep()
    s.vcycle(cycles)
    so, sg = o.state(), s.state()
    so["t_overlap"], so["t_overlap_old"] = o.overlap()
    sg["t_overlap"], sg["t_overlap_old"] = s.overlap()
    check_corrected(sg, so)
    assert float(np.linalg.norm(sg["res_L1"])) == pytest.approx(norms[-1], rel=1e-9)


@pytest.mark.gpu
def test_corrected_cycle_time_loop_and_schedules():
    """pamg_run with cycle = 1 (begin_timestep + cycles) equals the oracle over two steps; the
    fused switch is ignored (the corrected cycle runs the per-step kernels)."""
    import pamg
    om = O.read_msh(os.path.join(goldens.MESHES, "irregular.msh"))
    o = O.Oracle(om, 4, 3, ntime=2, n_multigrid=2)
    for _ in range(2):
        o.begin_timestep()
        for _ in range(2):
            o.vcycle_corrected()
    m = pamg.Mesh.read(os.path.join(goldens.MESHES, "irregular.msh"))
    for fused in (0, 3):
        s = pamg.SemiImplicitIterative(m, 4, 3, cycle=1, fused=fused)
        s.run(2, 2)
        check_corrected(s.state(), o.state())


# ---------------------------------------------------------------- the resident corrected call
def corr_pair(mesh, S, L, arith, solver=3, ns=4, fused=3):
    """the HIP path (cycle = 1) and the oracle in the same arithmetic, the oracle taking the device's
    source term s' (the one operation the two sides cannot share, tests/test_contracted_oracle.py)"""
    import pamg
    path = os.path.join(goldens.MESHES, mesh)
    g = pamg.SemiImplicitIterative(pamg.Mesh.read(path), S, L, n_smooth=ns, solver=solver, fused=fused, arith=arith,
                                   cycle=1)
    o = O.Oracle(O.read_msh(path), S, L, n_smooth=ns, solver=solver, arith=arith)
    o.set_source(g.get(pamg.SOURCE, 1))
    return g, o


def assert_identical(g, o):
    sg, so = g.state(), o.state()
    for k in so:
        np.testing.assert_array_equal(sg[k], so[k], err_msg=k)
    for x, y in zip(g.overlap(), o.overlap()):
        np.testing.assert_array_equal(x, y)


@pytest.mark.gpu
@pytest.mark.parametrize("arith", [1, 0])
def test_corrected_resident_call_is_bitwise_the_oracle_at_the_bench_config(arith):
    """bench.py's extra.cycle1 workload -- untitled8192, n_split 5, L 3, n_smooth 4, solver 3, one
    time step and a pamg_vcycle(4) call, i.e. ONE resident launch (k_vc_corr) -- is every field of
    every level, t_overlap and t_overlap_old of orc_vcycle_corrected's four cycles, bit for bit."""
    g, o = corr_pair("untitled8192.msh", 5, 3, arith)
    g.timing_enable(1 << 14)   # PAMG_K_VCYCLE_CORR
    g.timing_reset()
    g.begin_timestep()
    g.vcycle(4)
    o.begin_timestep()
    for _ in range(4):
        o.vcycle_corrected()
    assert g.timing()["vcycle_corr"]["issued"] == 1
    assert_identical(g, o)


@pytest.mark.gpu
@pytest.mark.parametrize("mesh,S,L,solver,ns", [
    ("untitled8.msh", 3, 3, 3, 4), ("irregular.msh", 6, 3, 1, 2), ("900_ele.msh", 2, 2, 3, 3),
    ("test_sn2.msh", 4, 4, 3, 2), ("untitled2048.msh", 5, 5, 3, 1), ("irregular.msh", 7, 4, 3, 2),
    ("untitled8192.msh", 3, 3, 1, 4), ("untitled8.msh", 1, 1, 3, 2)])
@pytest.mark.parametrize("arith", [1, 0])
def test_corrected_resident_call_equals_per_step_and_oracle(mesh, S, L, solver, ns, arith):
    """The resident call (fused = 3: whole-un_ele tiles below n_split 5, parts of one at 6 and 7, two to
    five levels, Jacobi and GS, calls split 2 + 1 over two time steps) and the per-step sequence
    (fused = 0) leave the oracle's state, bit for bit."""
    o = None
    for fused in (3, 0):
        g, o1 = corr_pair(mesh, S, L, arith, solver, ns, fused)
        for _ in range(2):
            g.begin_timestep()
            g.vcycle(2)
            g.vcycle(1)
        if o is None:
            o = o1
            for _ in range(2):
                o.begin_timestep()
                for _ in range(3):
                    o.vcycle_corrected()
        assert_identical(g, o)
        g.close()
