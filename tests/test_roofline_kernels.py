"""The level-1 roofline sweep kernels (bench.py `roofline_hbm_smoother`, `extra.sweep_*`) compute a sweep.

k_sweep_stencil (per-un_ele stencil, the reference's operation order) and k_sweep_assembled
(the assembled element-block-sparse operator of matrices.F90:997-1198 -- one 3x3 block and
omega/D per sub-element, 168 B per sub-element -- in the contracted arithmetic of arith = 1)
each run ONE Jacobi sweep of level 1 (solve_Jacobi, transport_tri_semi.F90:491-497) from
tnew_nonlin and RHS. Their outputs are compared with the oracle's orc_sweep_once, bit for bit,
on untitled8192 at the benchmarked n_split = 5 (8,388,608 sub-elements) and at n_split = 3;
orc_sweep_once itself is pinned to the oracle's smoother (which the reference goldens pin,
tests/test_oracle_golden.py) by the CPU tests below.
"""
import os

import numpy as np
import pytest

import goldens
import oracle_lib as O

TNEW, RHS, TNN = O.TNEW, O.RHS, O.TNN


def _random_state(shape, seed):
    rng = np.random.default_rng(seed)
    return rng.uniform(-1, 1, shape), rng.uniform(-1, 1, shape)


@pytest.mark.parametrize("arith", [0, 1])
@pytest.mark.parametrize("mesh,S", [("untitled8.msh", 3), ("irregular.msh", 3), ("900_ele.msh", 2)])
def test_oracle_sweep_once_is_one_smoother_sweep(mesh, S, arith):
    """orc_sweep_once(level 2) == the oracle's smoother with n_smooth = 1 on level 2 (level 2, so
    the smoother does not rebuild the RHS as it does on level 1, :593), both arithmetics"""
    m = O.read_msh(os.path.join(goldens.MESHES, mesh))
    o = O.Oracle(m, S, 2, n_smooth=1, arith=arith)
    x, b = _random_state((3, o.nsub(2), m.U), 7)
    o.set(TNEW, 2, x)
    o.copy_to_tnn(2)
    o.set(RHS, 2, b)
    o.smoother(2)
    np.testing.assert_array_equal(o.sweep_once(2, arith, x, b), o.get(TNN))


def test_oracle_sweep_once_arithmetics_agree():
    m = O.read_msh(os.path.join(goldens.MESHES, "untitled8.msh"))
    o = O.Oracle(m, 3, 1)
    x, b = _random_state((3, o.nsub(1), m.U), 11)
    y0, y1 = o.sweep_once(1, 0, x, b), o.sweep_once(1, 1, x, b)
    assert goldens.rel_err(y1, y0) < 1e-13


@pytest.mark.gpu
@pytest.mark.parametrize("S", [3, 5])
def test_gpu_roofline_sweeps_match_oracle(S):
    import pamg
    path = os.path.join(goldens.MESHES, "untitled8192.msh")
    s = pamg.SemiImplicitIterative(pamg.Mesh.read(path), S, 1)
    o = O.Oracle(O.read_msh(path), S, 1)
    x, b = _random_state((3, s.nsub(1), s.U), 20251015 + S)
    s.set(pamg.TNEW_NONLIN, 1, x)
    s.set(pamg.RHS, 1, b)
    got0 = s.sweep_bench_output(False)
    np.testing.assert_array_equal(got0, o.sweep_once(1, 0, x, b))
    got1 = s.sweep_bench_output(True)
    np.testing.assert_array_equal(got1, o.sweep_once(1, 1, x, b))
    # the two operation orders are one sweep of the same operator
    assert goldens.rel_err(got1, got0) < 1e-13
    # the kernels read only tnew_nonlin and RHS: the state is untouched
    np.testing.assert_array_equal(s.get(pamg.TNEW_NONLIN, 1), x)
    np.testing.assert_array_equal(s.get(pamg.RHS, 1), b)
    # and the timed launches are the same kernels (they run and report their 168 / 72 B per sub-element)
    ms_a, by_a = s.sweep_bench(3, True)
    ms_s, by_s = s.sweep_bench(3, False)
    N = s.U * 4 ** S
    assert ms_a > 0 and ms_s > 0 and by_a == 168.0 * N and by_s == 72.0 * N + 168.0 * s.U
    s.close()
