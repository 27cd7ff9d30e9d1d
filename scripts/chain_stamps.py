"""Phase timeline of the persistent face chain (PAMG_CHAIN_STAMPS): per launch, the mean per-sweep
wait / passes / publish time of workgroups 0..7 (wall clock 100 MHz); for the per-wave chain
(k_face_chain_pw, a negative run in the header) every wave's phases: item-0 pass, wait, snapshot,
item-1 pass with its words + drain + flag, down pass, the rest. usage: chain_stamps.py FILE"""
import sys

import numpy as np

raw = np.fromfile(sys.argv[1], np.int64)
i = 0
while i < raw.size:
    run, grid, E, nsub = (int(v) for v in raw[i:i + 4])
    i += 4
    if run < 0:   # per-wave: [8 workgroups][16 waves][run][7]
        run = -run
        st = raw[i:i + 8 * 16 * run * 7].reshape(8 * 16, run, 7).astype(np.float64) * 10e-3
        i += 8 * 16 * run * 7
        st = st[:min(8, grid) * 16]
        if run < 4:
            continue
        s = st[:, 1:-1]   # steady sweeps (the first has no wait, the last no words)
        names = ["item0", "wait", "snap", "item1", "drain+flag", "downs"]
        ph = [(s[:, :, k + 1] - s[:, :, k]).mean() for k in range(6)]
        rest = (st[:, 2:, 0] - st[:, 1:-1, 6]).mean()
        per = (st[:, -1, 0] - st[:, 1, 0]).mean() / (run - 2)
        # the sweep's critical hand-off: the last flag of sweep sw among these waves -> the first wait end of sw + 1
        fl = st[:, 1:-2, 5].max(axis=0)
        we = st[:, 2:-1, 2]
        print(f"pw run {run:3d} grid {grid:4d}: per sweep {per:6.2f} us = " +
              " + ".join(f"{n} {v:5.2f}" for n, v in zip(names, ph)) + f" + rest {rest:5.2f}; "
              f"wait end - last flag (these waves): min {(we.min(axis=0) - fl).mean():5.2f} "
              f"mean {(we.mean(axis=0) - fl).mean():5.2f} us; flag spread {(st[:, 1:-1, 5].max(0) - st[:, 1:-1, 5].min(0)).mean():5.2f} us")
        continue
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
