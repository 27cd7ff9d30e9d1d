"""csr_mul_array (matrices.F90:172-193), the north star's "matrices.F90 SpMV".

Fixture: tests/golden/csr.npz -- matrices in the reference's `type sparse` storage
multiplied by the reference's own csr_mul_array (oracle/build_ref.py -> csr_ref_fp64,
tests/make_golden_csr.py): random 3-per-row matrices, boundary rows with repeated
columns, the reference's P1 mass matrices in its global numbering, and a 9-per-row
matrix of which the routine reads only the first 3 nrows entries. The oracle
restatement, the HIP kernel (C-ABI and the Fortran drop-in) reproduce it bit for bit.
"""
import json
import os
import subprocess

import numpy as np
import pytest

import goldens
import oracle_lib as O

FIX = np.load(os.path.join(goldens.GOLDEN, "csr.npz"), allow_pickle=False)
META = json.loads(str(FIX["meta"]))
CASES = [m["case"] for m in META]


def case(k):
    return {n: FIX[f"c{k}_{n}"] for n in ("iloc", "jloc", "val", "array", "result")}


@pytest.mark.parametrize("k", CASES)
def test_oracle_csr_matches_reference(k):
    c = case(k)
    got = O.csr_mul_array(c["iloc"].size, c["jloc"], c["val"], c["array"])
    np.testing.assert_array_equal(got, c["result"])


def test_fixture_covers_the_quirks():
    kinds = {m["kind"]: m for m in META}
    assert {"random", "repeated", "mass_u8_s3", "nine_per_row"} <= set(kinds)
    k = kinds["nine_per_row"]["case"]
    c = case(k)
    n = c["iloc"].size
    # the routine reads entries 1 .. 3 nrows in storage order, whatever g_iloc says
    v, j = c["val"][:3 * n].reshape(n, 3), c["jloc"][:3 * n].reshape(n, 3) - 1
    ref = ((0.0 + v[:, 0] * c["array"][j[:, 0]]) + v[:, 1] * c["array"][j[:, 1]]) + v[:, 2] * c["array"][j[:, 2]]
    np.testing.assert_array_equal(ref, c["result"])


@pytest.mark.gpu
@pytest.mark.parametrize("k", CASES)
def test_gpu_csr_matches_reference(k):
    import pamg
    s = pamg.SemiImplicitIterative(pamg.Mesh.read(os.path.join(goldens.MESHES, "untitled8.msh")), 1, 1)
    c = case(k)
    got = pamg.csr_mul_array(s, (c["iloc"], c["jloc"], c["val"]), c["array"])
    np.testing.assert_array_equal(got, c["result"])


@pytest.mark.gpu
def test_gpu_csr_full_size_against_oracle():
    """The assembled level-1 operator's size at n_split = 5 on untitled8192: 25.2 M rows of
    the reference's block numbering; vs the oracle, bitwise. (pamg_csr_mul_array stages the
    vectors and runs the device entry point pamg_csr_mul_array_device.)"""
    import pamg
    s = pamg.SemiImplicitIterative(pamg.Mesh.read(os.path.join(goldens.MESHES, "untitled8.msh")), 1, 1)
    rng = np.random.default_rng(20251015)
    nrows = 3 * 8192 * 4 ** 5
    base = 3 * (np.arange(nrows, dtype=np.int32) // 3)
    jloc = (base[:, None] + np.arange(1, 4, dtype=np.int32)[None, :]).reshape(-1)
    val = rng.uniform(-1, 1, 3 * nrows)
    x = rng.uniform(-1, 1, nrows)
    iloc = np.arange(1, 3 * nrows, 3, dtype=np.int32)
    ref = O.csr_mul_array(nrows, jloc, val, x)
    m = pamg.Sparse(s, iloc, jloc, val)
    np.testing.assert_array_equal(m.mul_array(x), ref)
    np.testing.assert_array_equal(m.mul_array(-x), -ref)   # staging buffers reused
    m.close()


def test_csr_rejects_short_rows():
    """nnz < 3 nrows would make the reference read past val (matrices.F90:187): an error."""
    import pamg
    if not os.path.exists("/dev/kfd"):
        pytest.skip("needs a handle (GPU)")
    s = pamg.SemiImplicitIterative(pamg.Mesh.read(os.path.join(goldens.MESHES, "untitled8.msh")), 1, 1)
    with pytest.raises(pamg.PamgError):
        pamg.Sparse(s, np.arange(1, 10, 3), np.ones(8, np.int32), np.ones(8))


@pytest.mark.gpu
@pytest.mark.parametrize("k", CASES)
def test_fortran_csr_dropin_matches_reference(tmp_path, k):
    exe = os.path.join(os.path.dirname(goldens.HERE), "p-a_multigrids_amd", "bin", "csr_host")
    c = case(k)
    with open(tmp_path / "csr_in.bin", "wb") as f:
        np.array([c["iloc"].size, c["jloc"].size, c["array"].size], np.int32).tofile(f)
        c["iloc"].astype(np.int32).tofile(f)
        c["jloc"].astype(np.int32).tofile(f)
        c["val"].astype(np.float64).tofile(f)
        c["array"].astype(np.float64).tofile(f)
    r = subprocess.run([exe], cwd=tmp_path, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    np.testing.assert_array_equal(np.fromfile(tmp_path / "csr_out.bin", np.float64), c["result"])
