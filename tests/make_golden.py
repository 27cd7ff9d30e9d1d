#!/usr/bin/env python3
"""Generate tests/golden/*.npz from the instrumented reference build.

Runs oracle/_ref/pamg_ref_{fp64,fp32} (built by oracle/build_ref.py from the
reference sources under /root/reference) on the meshes in tests/meshes with a
pamg_ref.nml configuration, and stores the binary state dumps it writes
(oracle/ref_hooks/pamg_ref_hooks.F90) as compressed numpy archives. The
reference's own tests hold no known-answer data for this path (SURVEY.md
section 4), so these vectors are the parity pin. Only data is committed: inputs
(the .msh files) and the reference's outputs.

Usage: python tests/make_golden.py [--only NAME]
"""
import argparse
import json
import os
import re
import shutil
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, HERE)
import pamg_records  # noqa: E402

REF_DIR = os.path.join(ROOT, "oracle", "_ref")
GOLDEN = os.path.join(HERE, "golden")

# name: (mesh, n_split, levels, n_smooth, solver, ntime, n_multigrid, dump_calls, precision, sample)
CASES = {
    "u8_s1_l1_plumbing":   ("untitled8.msh", 1, 1, 4, 3, 1, 1, 0, "fp64", None),
    "u8_s3_l3_gs":         ("untitled8.msh", 3, 3, 4, 3, 2, 2, 1, "fp64", None),
    "u8_s3_l3_jacobi":     ("untitled8.msh", 3, 3, 4, 1, 2, 2, 0, "fp64", None),
    "u8_s2_l2_richardson": ("untitled8.msh", 2, 2, 4, 2, 2, 2, 1, "fp64", None),
    "u8_s3_l3_gs_fp32":    ("untitled8.msh", 3, 3, 4, 3, 2, 2, 0, "fp32", None),
    "u8_s2_l2_smooth1":    ("untitled8.msh", 2, 2, 1, 3, 2, 2, 0, "fp64", None),
    "sn2_default":         ("test_sn2.msh", 1, 1, 4, 3, 2, 2, 0, "fp64", None),
    "sn2_s3_l2":           ("test_sn2.msh", 3, 2, 3, 3, 2, 2, 0, "fp64", None),
    "two_unele_s4_l3":     ("2_unele_test.msh", 4, 3, 4, 3, 1, 2, 0, "fp64", None),
    "irregular_s3_l3":     ("irregular.msh", 3, 3, 4, 3, 2, 2, 0, "fp64", None),
    "e900_s2_l2_jacobi":   ("900_ele.msh", 2, 2, 4, 1, 1, 2, 0, "fp64", None),
    "u8192_s3_l3_1cycle":  ("untitled8192.msh", 3, 3, 4, 3, 1, 1, 0, "fp64", 16384),
    # the benchmarked instances: the bench workload's own shape (S = 5, the resident
    # k_vc_resb tiles), config 5's mesh at S = 6 (sub-un_ele tiles) and config 2's exact shape
    "u8192_s5_l3":         ("untitled8192.msh", 5, 3, 4, 3, 1, 2, 0, "fp64", 32768),
    "irregular_s6_l3":     ("irregular.msh", 6, 3, 4, 3, 1, 2, 0, "fp64", None),
    "e900_s3_l3_jacobi":   ("900_ele.msh", 3, 3, 4, 1, 1, 2, 0, "fp64", None),
}


def run_case(name, spec):
    mesh, S, L, ns, solver, ntime, nmg, calls, prec, sample = spec
    exe = os.path.join(REF_DIR, f"pamg_ref_{prec}")
    if not os.path.exists(exe):
        raise SystemExit(f"{exe} missing: run python oracle/build_ref.py first")
    tmp = tempfile.mkdtemp(prefix="pamg_golden_")
    try:
        shutil.copy(os.path.join(HERE, "meshes", mesh), tmp)
        with open(os.path.join(tmp, "pamg_ref.nml"), "w") as f:
            f.write("&pamg_ref\n")
            f.write(f" pamg_mesh='{mesh}', pamg_dump_prefix='g', pamg_nsplit={S}, pamg_ntime={ntime},\n")
            f.write(f" pamg_nmultigrid={nmg}, pamg_solver={solver}, pamg_levels={L}, pamg_nsmooth={ns},\n")
            f.write(f" pamg_vtk=100000, pamg_dump_calls={calls}\n/\n")
        r = subprocess.run([exe], cwd=tmp, capture_output=True, text=True, timeout=3600)
        if r.returncode != 0:
            raise SystemExit(f"{name}: reference failed\n{r.stdout}\n{r.stderr}")
        m = re.search(r"cpu_time for time_loop =\s*([0-9.Ee+-]+)", r.stdout)
        t_loop = float(m.group(1)) if m else None
        arrays = {}
        final = pamg_records.read_records(os.path.join(tmp, "g_final.bin"))
        for k, v in final.items():
            arrays[k] = v
        for fn in sorted(os.listdir(tmp)):
            mm = re.match(r"g_call(\d+)_(\w+)_L(\d+)\.bin$", fn)
            if mm:
                tag = f"call{mm.group(1)}_{mm.group(2)}_L{mm.group(3)}"
                for k, v in pamg_records.read_records(os.path.join(tmp, fn)).items():
                    arrays[f"{tag}/{k}"] = v
        meta = dict(name=name, mesh=mesh, n_split=S, levels=L, n_smooth=ns, solver=solver, ntime=ntime,
                    n_multigrid=nmg, precision=prec, reference_time_loop_s=t_loop)
        if sample:
            # keep topology/geometry complete; sample the state arrays (every k-th value) + norms
            out = {}
            for k, v in arrays.items():
                if k.split("/")[-1].split("_L")[0] in ("tnew", "told", "RHS", "res", "tnew_nonlin", "t_overlap",
                                                       "t_overlap_old") and v.size > sample:
                    flat = v.reshape(-1, order="F")
                    step = max(1, flat.size // sample)
                    out[k + "@sample"] = flat[::step].copy()
                    out[k + "@step"] = np.array(step)
                    out[k + "@shape"] = np.array(v.shape)
                    out[k + "@l2"] = np.array(np.linalg.norm(flat))
                    out[k + "@max"] = np.array(flat.max())
                    out[k + "@min"] = np.array(flat.min())
                    out[k + "@sum"] = np.array(flat.sum())
                elif k.split("_L")[0] in ("mass", "kdiff", "ml", "detwei"):
                    continue  # geometry of 8192 elements is re-derived and pinned on smaller meshes
                else:
                    out[k] = v
            arrays = out
            meta["sampled"] = sample
        arrays["meta"] = np.array(json.dumps(meta))
        os.makedirs(GOLDEN, exist_ok=True)
        np.savez_compressed(os.path.join(GOLDEN, name + ".npz"), **arrays)
        print(f"{name}: {len(arrays)} arrays, time_loop={t_loop}")
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default=None)
    a = ap.parse_args()
    for name, spec in CASES.items():
        if a.only and a.only != name:
            continue
        run_case(name, spec)


if __name__ == "__main__":
    main()
