#!/usr/bin/env python3
"""Golden vectors of the reference's csr_mul_array (matrices.F90:172-193), the
matrices.F90 SpMV of the north star, computed by the reference's own routine
(oracle/_ref/csr_ref_fp64, oracle/build_ref.py; fp64 default real).

The routine walks the entries in storage order, 3 per row, for size(g_iloc) rows,
and never reads g_iloc's values: result(r) = ((0 + v(3r-2) a(j(3r-2))) + ...). Cases
(seed 20251015): random 3-per-row matrices (1 to 4,096 rows, columns anywhere,
repeated columns as at a domain boundary, :1084-1110), the P1 mass matrices of the
reference itself in its global numbering glob = 3 4**S (u-1) + 3 (s-1) + i
(matrices.F90:1496-1500; the element blocks of tests/golden/u8_s3_l3_gs.npz), and a
9-per-row flux-sized matrix, of which the routine consumes only the first 3 nrows
entries. Writes tests/golden/csr.npz (data only).
"""
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
EXE = os.path.join(ROOT, "oracle", "_ref", "csr_ref_fp64")
sys.path.insert(0, HERE)
import goldens  # noqa: E402


def run_ref(iloc, jloc, val, arr):
    with tempfile.TemporaryDirectory() as tmp:
        with open(os.path.join(tmp, "csr_in.bin"), "wb") as f:
            np.array([iloc.size, jloc.size, arr.size], np.int32).tofile(f)
            iloc.astype(np.int32).tofile(f)
            jloc.astype(np.int32).tofile(f)
            val.astype(np.float64).tofile(f)
            arr.astype(np.float64).tofile(f)
        r = subprocess.run([EXE], cwd=tmp, capture_output=True, text=True, timeout=300)
        if r.returncode != 0:
            raise SystemExit(r.stdout + r.stderr)
        return np.fromfile(os.path.join(tmp, "csr_out.bin"), np.float64)


def cases(rng):
    out = []
    for nrows, n in ((1, 1), (1, 5), (7, 3), (64, 200), (1000, 3000), (4096, 12288)):
        jloc = rng.integers(1, n + 1, 3 * nrows)
        out.append(("random", np.arange(1, 3 * nrows, 3), jloc, rng.uniform(-1, 1, 3 * nrows),
                    rng.uniform(-1, 1, n)))
    nrows, n = 500, 1500   # boundary rows: the self columns repeated
    jloc = np.repeat(rng.integers(1, n + 1, nrows), 3)
    out.append(("repeated", np.arange(1, 3 * nrows, 3), jloc, rng.uniform(-1e3, 1e3, 3 * nrows),
                rng.uniform(-1e-6, 1e-6, n)))
    meta, d = goldens.load("u8_s3_l3_gs")   # the reference's own element mass matrices
    M = d["mass_L1"]                          # (3, 3, U): one block per un_ele at level 1
    U, nsub = M.shape[-1], 4 ** meta["n_split"]
    rows, cols, vals = [], [], []
    for u in range(U):
        for s in range(nsub):
            base = 3 * nsub * u + 3 * s
            for i in range(3):
                for j in range(3):
                    rows.append(base + i)
                    cols.append(base + j + 1)
                    vals.append(M[i, j, u])
    n = 3 * nsub * U
    out.append(("mass_u8_s3", np.arange(1, n * 3, 3), np.array(cols), np.array(vals), rng.uniform(-1, 1, n)))
    nrows, n = 300, 900    # 9 entries per row (the flux matrix's size); the routine reads 3 per row
    out.append(("nine_per_row", np.arange(1, 9 * nrows, 9), rng.integers(1, n + 1, 9 * nrows),
                rng.uniform(-1, 1, 9 * nrows), rng.uniform(-1, 1, n)))
    return out


def main():
    rng = np.random.default_rng(20251015)
    arrays, meta = {}, []
    for k, (kind, iloc, jloc, val, arr) in enumerate(cases(rng)):
        res = run_ref(iloc, jloc, val, arr)
        assert res.size == iloc.size
        for name, a in (("iloc", iloc), ("jloc", jloc), ("val", val), ("array", arr), ("result", res)):
            arrays[f"c{k}_{name}"] = np.asarray(a, np.int32 if name in ("iloc", "jloc") else np.float64)
        meta.append(dict(case=k, kind=kind, nrows=int(iloc.size), nnz=int(jloc.size), n=int(arr.size)))
        print(k, kind, iloc.size, jloc.size, arr.size)
    arrays["meta"] = np.array(json.dumps(meta))
    np.savez_compressed(os.path.join(HERE, "golden", "csr.npz"), **arrays)


if __name__ == "__main__":
    main()
