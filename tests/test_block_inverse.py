"""FINDInv (matrix_inversion.F90:50-148), the north star's "local block solve", and the
direct path built on it (coarse_solver = 1).

Fixture: tests/golden/findinv.npz -- batches of n x n matrices (n = 1..8) inverted by the
reference's own FINDInv compiled unmodified (oracle/build_ref.py -> findinv_ref_fp64,
tests/make_golden_findinv.py), including its zero-pivot row repair, its early give-up and
singular inputs. The oracle restatement and the HIP kernel must reproduce it bit for bit.
The direct coarse solve has no reference output (the reference's mode 9 does not use it):
it is pinned to the oracle restatement, whose FINDInv is pinned here.
"""
import os

import numpy as np
import pytest

import goldens
import oracle_lib as O

FIX = np.load(os.path.join(goldens.GOLDEN, "findinv.npz"), allow_pickle=False)
NS = (1, 2, 3, 4, 6, 8)


def same(a, b):
    return np.array_equal(a, b, equal_nan=True)


@pytest.mark.parametrize("n", NS)
def test_oracle_findinv_matches_reference(n):
    A, inv, err = FIX[f"n{n}_A"], FIX[f"n{n}_inv"], FIX[f"n{n}_err"]
    got, gerr = O.findinv(A)
    np.testing.assert_array_equal(gerr, err)
    assert same(got, inv)


def test_fixture_covers_the_quirks():
    # the zero-pivot repair, the early give-up and genuine singular matrices are all present
    assert (FIX["n3_err"] == -1).sum() >= 5 and (FIX["n3_err"] == 0).sum() > 1000
    A = FIX["n4_A"]
    assert any(A[0, 0, q] == 0 and FIX["n4_err"][q] == 0 for q in range(A.shape[2]))   # repaired
    assert any(A[0, 0, q] == 0 and A[1, 0, q] == 0 and np.linalg.matrix_rank(A[:, :, q]) == 4 and
               FIX["n4_err"][q] == -1 for q in range(A.shape[2]))                     # given up


def test_direct_coarse_solve_solves_the_block_system():
    """Oracle direct path: A_e x = b to rounding on the coarsest level after a V-cycle."""
    mesh = O.read_msh(os.path.join(goldens.MESHES, "untitled8.msh"))
    o = O.Oracle(mesh, 3, 3, ntime=1, n_multigrid=1, coarse_solver=1)
    o.run()
    _, M, Kd, _ = o.geometry(3)
    x, b = o.get(O.TNEW, 3), o.get(O.RHS, 3)
    A = M / 1.25e-5 + Kd
    r = np.einsum("iju,jsu->isu", A, x) - b
    assert np.abs(r).max() <= 1e-12 * max(np.abs(b).max(), 1e-300)


@pytest.mark.gpu
@pytest.mark.parametrize("n", NS)
def test_gpu_block_inverse_matches_reference(n):
    import pamg
    mesh = pamg.Mesh.read(os.path.join(goldens.MESHES, "untitled8.msh"))
    s = pamg.SemiImplicitIterative(mesh, 1, 1)
    A, inv, err = FIX[f"n{n}_A"], FIX[f"n{n}_inv"], FIX[f"n{n}_err"]
    got, gerr = s.block_inverse(A)
    np.testing.assert_array_equal(gerr, err)
    assert same(got, inv)


@pytest.mark.gpu
@pytest.mark.parametrize("mesh_name,S,L", [("untitled8.msh", 3, 3), ("900_ele.msh", 2, 2),
                                           ("untitled8192.msh", 3, 3)])
def test_gpu_direct_coarse_solve_matches_oracle(mesh_name, S, L):
    import pamg
    path = os.path.join(goldens.MESHES, mesh_name)
    s = pamg.SemiImplicitIterative(pamg.Mesh.read(path), S, L, coarse_solver=1)
    s.run(2, 2)
    o = O.Oracle(O.read_msh(path), S, L, ntime=2, n_multigrid=2, coarse_solver=1)
    o.run()
    got, ref = s.state(), o.state()
    for k, v in ref.items():
        assert goldens.rel_err(got[k], v) <= 1e-10, k


@pytest.mark.gpu
@pytest.mark.parametrize("n", (3, 6))
def test_fortran_findinv_dropin_matches_reference(tmp_path, n):
    """`use matrix_inversion; call FINDInv(a, inv, n, ierr)` as at a reference call site,
    answered by the GPU (p-a_multigrids_amd/fortran/matrix_inversion.F90)."""
    import subprocess
    exe = os.path.join(os.path.dirname(goldens.HERE), "p-a_multigrids_amd", "bin", "findinv_host")
    A, inv, err = FIX[f"n{n}_A"], FIX[f"n{n}_inv"], FIX[f"n{n}_err"]
    cnt = A.shape[2]
    with open(tmp_path / "findinv_in.bin", "wb") as f:
        np.array([n, cnt], np.int32).tofile(f)
        np.asfortranarray(A).reshape(-1, order="F").tofile(f)
    r = subprocess.run([exe], cwd=tmp_path, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    raw = (tmp_path / "findinv_out.bin").read_bytes()
    got = np.frombuffer(raw[:8 * n * n * cnt], np.float64).reshape((n, n, cnt), order="F")
    gerr = np.frombuffer(raw[8 * n * n * cnt:], np.int32)
    np.testing.assert_array_equal(gerr, err)
    assert same(got, inv)
    assert r.stdout.count("Matrix is non - invertible") == int((err != 0).sum())
