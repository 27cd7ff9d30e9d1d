"""Phase timeline of the persistent face chain (PAMG_CHAIN_STAMPS): per launch, the mean per-sweep
wait / passes / publish time of workgroups 0..7 (wall clock 100 MHz). usage: chain_stamps.py FILE"""
import sys

import numpy as np

raw = np.fromfile(sys.argv[1], np.int64)
i = 0
while i < raw.size:
    run, grid, E, nsub = (int(v) for v in raw[i:i + 4])
    i += 4
    st = raw[i:i + 8 * run * 4].reshape(8, run, 4).astype(np.float64) * 10e-3   # 100 MHz -> us
    i += 8 * run * 4
    w = min(8, grid)
    st = st[:w]
    wait = (st[:, 1:, 1] - st[:, 1:, 0]).mean()
    comp = (st[:, :, 2] - st[:, :, 1]).mean()
    pub = (st[:, :, 3] - st[:, :, 2]).mean()
    per = (st[:, -1, 3] - st[:, 0, 0]).mean() / run
    print(f"run {run:3d} grid {grid:4d} E {E:5d} nsub {nsub:5d}: per sweep {per:6.2f} us = wait {wait:5.2f} + passes "
          f"{comp:5.2f} + publish {pub:5.2f}")
