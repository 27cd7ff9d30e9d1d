"""Phase timeline of the face operator's wavefront calls (PAMG_WAVE_STAMPS): per launch, the grid
and, over workgroups 0..7's tickets, the mean time per ticket and per phase (wall clock 100 MHz).
usage: wave_stamps.py FILE"""
import sys

import numpy as np

T, W = 32, 19
raw = np.fromfile(sys.argv[1], np.int64)
i = 0
while i < raw.size:
    run, grid, U, nsub = (int(v) for v in raw[i:i + 4])
    i += 4
    st = raw[i:i + 8 * T * W].reshape(8, T, W).astype(np.float64) * 10e-3   # -> us
    i += 8 * T * W
    ok = st[:, :, 0] > 0
    tk = st[ok]
    if not len(tk):
        continue
    tot = (tk[:, W - 1] - tk[:, 0]).mean()
    load = (tk[:, 1] - tk[:, 0]).mean()
    ph = []
    for sw in range(min(run, 4)):
        k = 2 + 4 * sw
        prev = tk[:, 1] if sw == 0 else tk[:, k - 1]
        ph.append("s%d wait %.2f snap %.2f pass %.2f pub %.2f" % (
            sw, (tk[:, k] - prev).mean(), (tk[:, k + 1] - tk[:, k]).mean(), (tk[:, k + 2] - tk[:, k + 1]).mean(),
            (tk[:, k + 3] - tk[:, k + 2]).mean()))
    span = (st[:, :, W - 1].max() - st[:, :, 0][ok].min())
    print(f"run {run} grid {grid} U {U} nsub {nsub}: tickets/wg {ok.sum(1).mean():.1f}, per ticket {tot:.2f} us "
          f"(load {load:.2f}; {'; '.join(ph)}), wg0-7 span {span:.1f} us")
