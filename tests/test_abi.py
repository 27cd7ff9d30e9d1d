"""CPU checks of the C-ABI boundary: libpamg.so loads, exports every entry point
include/pamg.h declares, and refuses to run without a GPU instead of falling
back to a CPU path."""
import ctypes as C
import os
import re

import pytest

import pamg
from pamg import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "pamg.h")


def header_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(pamg_\w+)\s*\(", text)))


def test_header_declares_the_hot_path():
    fns = header_functions()
    for name in ("pamg_smoother", "pamg_restrictor", "pamg_get_residual", "pamg_prolongator",
                 "pamg_vcycle", "pamg_begin_timestep", "pamg_upload_mesh", "pamg_comm_init"):
        assert name in fns


def test_library_exports_every_declared_symbol():
    L = _lib.lib()
    missing = [f for f in header_functions() if not hasattr(L, f)]
    assert not missing, missing


def test_python_binding_covers_every_declared_symbol():
    src = open(os.path.join(ROOT, "p-a_multigrids_amd", "pamg", "_lib.py")).read()
    missing = [f for f in header_functions() if f'"{f}"' not in src]
    assert not missing, missing


def test_version_and_defaults_match_reference_mode9():
    L = _lib.lib()
    assert L.pamg_version() >= 100
    p = pamg.default_params()
    # main.F90:46-47 and transport_tri_semi.F90:117-140
    assert (p.n_split, p.multi_levels, p.n_smooth, p.n_coarse, p.solver) == (1, 1, 4, 15, 3)
    assert p.dt == 1.0 * 0.0000125 and p.k == 1.0 and p.omega == 0.8 and p.theta == 1.0


def test_parameter_validation():
    L = _lib.lib()
    h = C.c_void_p()
    bad = [dict(multi_levels=3, n_split=2), dict(theta=0.5), dict(solver=4), dict(dt=0.0)]
    for kw in bad:
        p = pamg.default_params(**kw)
        assert L.pamg_create(C.byref(p), C.byref(h)) == -1, kw


@pytest.mark.skipif(os.path.exists("/dev/kfd"), reason="a GPU may be present")
def test_no_gpu_fails_loudly():
    """Without a device the product path refuses to run (no CPU fallback)."""
    p = pamg.default_params()
    h = C.c_void_p()
    rc = _lib.lib().pamg_create(C.byref(p), C.byref(h))
    assert rc == -6   # PAMG_ERR_NODEV
    with pytest.raises(pamg.PamgError):
        pamg.SemiImplicitIterative(pamg.Mesh.read(os.path.join(ROOT, "tests", "meshes", "untitled8.msh")), 1, 1)


@pytest.mark.gpu
def test_c_host_example_runs_the_time_loop():
    """examples/c_host (plain C against include/pamg.h, the shape of a cgo / JNI stub)
    runs the mode-9 time loop; its |tnew_L1|^2 equals the oracle's to 1e-12."""
    import subprocess

    import numpy as np

    import goldens
    import oracle_lib as O
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    mesh = os.path.join(goldens.MESHES, "untitled8.msh")
    r = subprocess.run([os.path.join(root, "examples", "c_host"), mesh, "3", "3"], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    got = float(r.stdout.split("|tnew_L1|^2=")[1].split()[0])
    o = O.Oracle(O.read_msh(mesh), 3, 3, ntime=2, n_multigrid=2)
    o.run()
    ref = float(np.sum(o.get(O.TNEW, 1) ** 2))
    assert abs(got - ref) <= 1e-12 * ref
    assert "destroyed" in r.stdout


def test_every_runtime_switch_is_tested_or_diagnostics_only():
    """every PAMG_* environment switch compiled into the default libpamg is exercised by
    a test (tests/*.py names it); the diagnostics (stamps, halo-dropping A/B) are compiled in only with the
    PAMG_STAMPS build (`PAMG_STAMPS ? getenv(..) : nullptr`, `PAMG_STAMPS && getenv(..)`)."""
    import glob
    import re
    csrc = os.path.join(ROOT, "p-a_multigrids_amd", "csrc")
    tests = "".join(open(f).read() for f in glob.glob(os.path.join(ROOT, "tests", "*.py"))
                    if not f.endswith("test_abi.py"))
    untested = []
    for f in sorted(glob.glob(os.path.join(csrc, "*"))):
        for ln in open(f):
            for m in re.finditer(r'getenv\("(PAMG_[A-Z0-9_]+)"\)', ln):
                diag = re.search(r"PAMG_STAMPS\s*(\?|&&)\s*getenv", ln)
                if not diag and m.group(1) not in tests:
                    untested.append((os.path.basename(f), m.group(1)))
    assert not untested, untested
