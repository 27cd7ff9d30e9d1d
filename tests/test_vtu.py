"""VTU output (pamg_write_vtu) against the reference's own get_vtu files
(get_vtk_files.F90:10-165; fixtures from tests/make_golden_vtu.py).

The reference prints Tracer with F12.10, error / analytical with F10.7 and the
coordinates with F10.3, so the comparison is to half a unit of the last printed
digit; cells, offsets and types are exact. pamg_write_vtu writes fp64."""
import os
import tempfile

import numpy as np
import pytest

import goldens
import vtu_io

CASES = ["vtu_u8_s2_l2", "vtu_irregular_s3_l3"]


def load(name):
    z = np.load(os.path.join(goldens.GOLDEN, name + ".npz"), allow_pickle=False)
    import json
    return json.loads(str(z["meta"])), {k: z[k] for k in z.files if k != "meta"}


@pytest.mark.parametrize("name", CASES)
def test_reference_vtu_fixture_is_consistent(name):
    """CPU: the fixture's cells are the reference's numbering (3 DG nodes per sub-element,
    get_vtk_files.F90:108-124) and its analytical field is sin(x + y) of its points."""
    meta, d = load(name)
    n = d["tracer"].size
    assert d["points"].shape == (n, 3) and d["connectivity"].tolist() == list(range(n))
    assert d["offsets"].tolist() == list(range(3, n + 1, 3)) and set(d["types"].tolist()) == {5}
    # the points are printed with 3 decimals: sin(x + y) of them agrees to that rounding
    assert np.abs(np.sin(d["points"][:, 0] + d["points"][:, 1]) - d["analytical"]).max() < 2e-3


@pytest.mark.gpu
@pytest.mark.parametrize("ascii", [False, True])
@pytest.mark.parametrize("name", CASES)
def test_vtu_matches_reference(name, ascii):
    import pamg
    meta, d = load(name)
    m = pamg.Mesh.read(os.path.join(goldens.MESHES, meta["mesh"]))
    s = pamg.SemiImplicitIterative(m, meta["n_split"], meta["levels"])
    # the reference writes Tracer_<ntime>.vtu at the start of its last step (:301-311)
    s.run(meta["ntime"] - 1, meta["n_multigrid"])
    with tempfile.TemporaryDirectory() as tmp:
        path = os.path.join(tmp, "Tracer.vtu")
        s.write_vtu(path, ascii=ascii)
        v = vtu_io.read_vtu(path)
    assert v["n_points"] == d["tracer"].size and v["n_cells"] == d["offsets"].size
    np.testing.assert_array_equal(v["cells"]["connectivity"], d["connectivity"])
    np.testing.assert_array_equal(v["cells"]["offsets"], d["offsets"])
    np.testing.assert_array_equal(v["cells"]["types"], d["types"])
    assert np.abs(v["points"] - d["points"]).max() <= 5e-4 + 1e-12
    assert np.abs(v["point_data"]["Tracer"] - d["tracer"]).max() <= 5e-11 + 1e-16
    assert np.abs(v["point_data"]["error"] - d["error"]).max() <= 5e-8 + 1e-16
    assert np.abs(v["point_data"]["analytical"] - d["analytical"]).max() <= 5e-8 + 1e-16
    # and the full-precision content is the solver's own state
    t = s.get(pamg.TNEW, 1).reshape(-1, order="F")
    np.testing.assert_array_equal(v["point_data"]["Tracer"], t)
