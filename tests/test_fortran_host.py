"""The Fortran host (p-a_multigrids_amd/bin/pamg_transport): the reference's
mode-9 driver with its hot-path call sites bound to libpamg via iso_c_binding.
GPU tests compare its dumps with the reference's goldens; the CPU test checks
that without a GPU it stops with an error instead of computing anything."""
import os
import shutil
import subprocess

import pytest

import goldens
import pamg_records

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "p-a_multigrids_amd", "bin", "pamg_transport")


def run_host(tmp_path, meta, call_sites=1, facade=0, vtk=0):
    shutil.copy(os.path.join(goldens.MESHES, meta["mesh"]), tmp_path)
    (tmp_path / "pamg_run.nml").write_text(
        f"&transport mesh_file='{meta['mesh']}', n_split={meta['n_split']}, multi_levels={meta['levels']},\n"
        f" n_smooth={meta.get('n_smooth', 4)}, solver={meta.get('solver', 3)}, ntime={meta['ntime']},\n"
        f" n_multigrid={meta['n_multigrid']}, device=0, dump='out.bin', call_sites={call_sites},\n"
        f" facade_sweeps={facade}, vtk_interval={vtk} /\n")
    return subprocess.run([EXE], cwd=tmp_path, capture_output=True, text=True, timeout=300)


def test_host_binary_built():
    assert os.access(EXE, os.X_OK), "build() must produce the Fortran host"


@pytest.mark.skipif(os.path.exists("/dev/kfd"), reason="GPU node: covered by the gpu tests")
def test_host_stops_without_gpu(tmp_path):
    meta, _ = goldens.load("u8_s1_l1_plumbing")
    r = run_host(tmp_path, meta)
    assert r.returncode != 0
    assert "pamg_create failed" in r.stdout + r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["u8_s1_l1_plumbing", "u8_s3_l3_gs", "sn2_default", "e900_s2_l2_jacobi",
                                  "u8_s2_l2_richardson"])
@pytest.mark.parametrize("call_sites", [1, 0])
def test_host_matches_reference(tmp_path, name, call_sites):
    meta, d = goldens.load(name)
    r = run_host(tmp_path, meta, call_sites)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "cpu_time for time_loop" in r.stdout
    got = pamg_records.read_records(str(tmp_path / "out.bin"))
    for k, v in got.items():
        assert goldens.rel_err(v, d[k]) <= 1e-10, k


@pytest.mark.gpu
def test_linear_solvers_facade_runs(tmp_path):
    meta, _ = goldens.load("u8_s3_l3_gs")
    r = run_host(tmp_path, meta, 1, facade=3)
    assert r.returncode == 0, r.stdout + r.stderr


FACADE = os.path.join(ROOT, "p-a_multigrids_amd", "bin", "facade_host")


@pytest.mark.gpu
@pytest.mark.parametrize("mesh,S,L,it", [("untitled8.msh", 3, 3, 5), ("irregular.msh", 4, 2, 3),
                                         ("900_ele.msh", 2, 2, -1), ("untitled8.msh", 2, 1, 1)])
def test_gssolver_mesh_sd_facade_matches_oracle(tmp_path, mesh, S, L, it):
    """A reference-shaped Fortran caller (fortran/facade_host.F90) builds meshL(:) of the
    reference's type(mesh) from module structures, binds it and calls
    GSsolver_MeshSD(meshL, 1, it) with LinearSolvers.F90:719-733's signature (it = -1: the
    argument omitted, the reference's default size(meshL)/2). After it sweeps its
    tracer(1)%tnew and tnew_nonlin (read back as type(fields)) equal the oracle's smoother state
    after begin_timestep, tnew_nonlin := tnew and `it` sweeps, bit for bit (the oracle takes the
    device's source term s', tests/test_contracted_oracle.py)."""
    import numpy as np

    import oracle_lib as O
    out = str(tmp_path / "facade.bin")
    r = subprocess.run([FACADE, os.path.join(goldens.MESHES, mesh), str(S), str(L), "1", str(it), out],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    raw = np.fromfile(out, np.float64)
    U, nsub, lv, used = (int(v) for v in raw[:4])
    n = 3 * nsub * U
    tnew, tnn, rhs, src = (raw[4 + q * n:4 + (q + 1) * n].reshape((3, nsub, U), order="F") for q in range(4))
    assert lv == 1 and used == (it if it >= 0 else U // 2) and raw.size == 4 + 4 * n
    o = O.Oracle(O.read_msh(os.path.join(goldens.MESHES, mesh)), S, L, n_smooth=used)
    o.set_source(src)
    o.begin_timestep()
    o.copy_to_tnn(1)
    o.smoother(1)
    np.testing.assert_array_equal(tnew, o.get(O.TNEW, 1))
    np.testing.assert_array_equal(tnn, o.get(O.TNN, 1))
    np.testing.assert_array_equal(rhs, o.get(O.RHS, 1))


@pytest.mark.gpu
def test_host_vtu_call_site_matches_reference(tmp_path):
    """vtk_interval = 1: the host writes Tracer_<itime>.vtu at the reference's get_vtu call
    site (:301-311); the last one equals the reference's file (tests/test_vtu.py tolerances)."""
    import json

    import numpy as np

    import vtu_io
    z = np.load(os.path.join(goldens.GOLDEN, "vtu_u8_s2_l2.npz"), allow_pickle=False)
    meta = json.loads(str(z["meta"]))
    r = run_host(tmp_path, meta, 1, vtk=1)
    assert r.returncode == 0, r.stdout + r.stderr
    v = vtu_io.read_vtu(str(tmp_path / f"Tracer_{meta['ntime']}.vtu"))
    assert os.path.exists(tmp_path / "Tracer_1.vtu")
    assert np.abs(v["point_data"]["Tracer"] - z["tracer"]).max() <= 5e-11 + 1e-16
    assert np.abs(v["points"] - z["points"]).max() <= 5e-4 + 1e-12
