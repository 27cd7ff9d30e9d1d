#!/usr/bin/env python3
"""Golden vectors of the reference's VTU output (get_vtu, get_vtk_files.F90:10-165,
called at transport_tri_semi.F90:301-311) for tests/test_vtu.py.

Runs the instrumented reference build (oracle/_ref/pamg_ref_fp64, oracle/build_ref.py)
with vtk_interval = 1 and stores the arrays of the file it writes at the start of the
last time step (Tracer_<ntime>.vtu: the state after ntime - 1 steps, with the error
field of get_error, :302-304) as tests/golden/vtu_<name>.npz. Only data is committed.
Usage: python tests/make_golden_vtu.py
"""
import json
import os
import shutil
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, HERE)
import vtu_io  # noqa: E402

CASES = {"vtu_u8_s2_l2": ("untitled8.msh", 2, 2, 2, 2), "vtu_irregular_s3_l3": ("irregular.msh", 3, 3, 2, 2)}


def main():
    exe = os.path.join(ROOT, "oracle", "_ref", "pamg_ref_fp64")
    for name, (mesh, S, L, ntime, nmg) in CASES.items():
        tmp = tempfile.mkdtemp(prefix="pamg_vtu_")
        try:
            shutil.copy(os.path.join(HERE, "meshes", mesh), tmp)
            with open(os.path.join(tmp, "pamg_ref.nml"), "w") as f:
                f.write(f"&pamg_ref\n pamg_mesh='{mesh}', pamg_dump_prefix='', pamg_nsplit={S}, pamg_ntime={ntime},\n"
                        f" pamg_nmultigrid={nmg}, pamg_solver=3, pamg_levels={L}, pamg_nsmooth=4,\n"
                        f" pamg_vtk=1, pamg_dump_calls=0\n/\n")
            r = subprocess.run([exe], cwd=tmp, capture_output=True, text=True, timeout=600)
            if r.returncode != 0:
                raise SystemExit(f"{name}: reference failed\n{r.stdout}\n{r.stderr}")
            v = vtu_io.read_vtu(os.path.join(tmp, f"Tracer_{ntime}.vtu"))
            meta = dict(name=name, mesh=mesh, n_split=S, levels=L, ntime=ntime, n_multigrid=nmg,
                        note="the reference's ascii VTU: Tracer F12.10, error/analytical F10.7, points F10.3")
            np.savez_compressed(os.path.join(HERE, "golden", name + ".npz"), meta=np.array(json.dumps(meta)),
                                points=v["points"].astype(np.float64),
                                tracer=v["point_data"]["Tracer"].astype(np.float64),
                                error=v["point_data"]["error"].astype(np.float64),
                                analytical=v["point_data"]["analytical"].astype(np.float64),
                                connectivity=v["cells"]["connectivity"], offsets=v["cells"]["offsets"],
                                types=v["cells"]["types"])
            print(name, v["n_points"], v["n_cells"])
        finally:
            shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    main()
