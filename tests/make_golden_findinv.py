#!/usr/bin/env python3
"""Golden vectors of the reference's FINDInv (matrix_inversion.F90:50-148), the
local block solve of the north star: batches of n x n matrices inverted by the
reference's own routine (oracle/_ref/findinv_ref_fp64, built by
oracle/build_ref.py from the unmodified reference source, fp64 default real).

Cases per n in {1, 2, 3, 4, 6, 8} (seed 20251015): diagonally dominant and
general random matrices, zero leading pivots that the routine repairs by adding
a lower row (:75-86), zero pivots it gives up on although the matrix is
invertible (the early return at :87-92 when the next row is zero too),
singular matrices (-1, inverse 0, :97-102) and, for n = 3, the operator blocks
(1/dt) M + Kd of the mode-9 smoother for every un_ele and level of untitled8
(S = 3) and 900_ele (S = 2). Writes tests/golden/findinv.npz (data only).
"""
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
EXE = os.path.join(ROOT, "oracle", "_ref", "findinv_ref_fp64")
sys.path.insert(0, HERE)


def run_ref(mats):
    n = mats.shape[0]
    cnt = mats.shape[2]
    with tempfile.TemporaryDirectory() as tmp:
        with open(os.path.join(tmp, "findinv_in.bin"), "wb") as f:
            np.array([n, cnt], np.int32).tofile(f)
            np.asfortranarray(mats).reshape(-1, order="F").astype(np.float64).tofile(f)
        r = subprocess.run([EXE], cwd=tmp, capture_output=True, text=True, timeout=300)
        if r.returncode != 0:
            raise SystemExit(r.stdout + r.stderr)
        raw = open(os.path.join(tmp, "findinv_out.bin"), "rb").read()
    inv = np.frombuffer(raw[:8 * n * n * cnt], np.float64).reshape((n, n, cnt), order="F")
    err = np.frombuffer(raw[8 * n * n * cnt:], np.int32)
    return inv, err


def cases(n, rng):
    out = []
    for _ in range(64):   # diagonally dominant
        a = rng.uniform(-1, 1, (n, n))
        out.append(a + np.diag(np.sign(np.diag(a)) * (n + 1.0)))
    for _ in range(64):   # general
        out.append(rng.uniform(-1, 1, (n, n)))
    for _ in range(16):   # badly scaled
        out.append(rng.uniform(-1, 1, (n, n)) * 10.0 ** rng.uniform(-12, 12, (n, 1)))
    if n >= 2:
        for k in range(n - 1):   # zero pivot at (k, k) after elimination, repaired by a lower row
            a = rng.uniform(-1, 1, (n, n))
            a[k, :k + 1] = 0.0
            a[k, k] = 0.0
            out.append(a)
        a = np.eye(n)[::-1].copy()   # anti-diagonal permutation
        out.append(a)
    if n >= 3:   # zero pivot, next row zero in that column, a later row not: the early return
        a = rng.uniform(-1, 1, (n, n))
        a[0, 0] = 0.0
        a[1, 0] = 0.0
        out.append(a)
    for _ in range(4):   # singular: repeated row, zero column
        a = rng.uniform(-1, 1, (n, n))
        if n >= 2:
            a[-1] = a[0]
        else:
            a[0, 0] = 0.0
        out.append(a)
        b = rng.uniform(-1, 1, (n, n))
        b[:, n // 2] = 0.0
        out.append(b)
    out.append(np.zeros((n, n)))
    return np.stack(out, axis=2)


def operator_blocks():
    import oracle_lib as O
    blocks = []
    for mesh, S, L in (("untitled8.msh", 3, 3), ("900_ele.msh", 2, 2)):
        o = O.Oracle(O.read_msh(os.path.join(HERE, "meshes", mesh)), S, L, ntime=1, n_multigrid=1)
        for l in range(1, L + 1):
            _, M, Kd, _ = o.geometry(l)
            rdt = 1 / 1.25e-5
            for u in range(M.shape[2]):
                blocks.append(rdt * M[:, :, u] + Kd[:, :, u])
    return np.stack(blocks, axis=2)


def main():
    if not os.path.exists(EXE):
        raise SystemExit(f"{EXE} missing: python oracle/build_ref.py")
    rng = np.random.default_rng(20251015)
    d = {}
    for n in (1, 2, 3, 4, 6, 8):
        A = cases(n, rng)
        if n == 3:
            A = np.concatenate([A, operator_blocks()], axis=2)
        inv, err = run_ref(A)
        d[f"n{n}_A"], d[f"n{n}_inv"], d[f"n{n}_err"] = A, inv, err
        print(f"n={n}: {A.shape[2]} matrices, {int((err != 0).sum())} flagged singular")
    np.savez_compressed(os.path.join(HERE, "golden", "findinv.npz"), **d)


if __name__ == "__main__":
    main()
