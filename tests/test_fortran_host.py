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
