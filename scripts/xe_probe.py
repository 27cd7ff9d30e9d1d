"""The per-call exchange of one rank at config 4's N = 8 shape, through RCCL (GPU box only): a 32 x 16 x 2
strip (1,024 un_eles at n_split 5 -- a rank's share of untitled8192 on 8 GPUs) as a self-peer partition of
`--parts` x-strips (pamg_comm_init_self: the cut's words go through ncclSend / ncclRecv to this rank), in the
driver's call shape (a fresh handle, begin_timestep, a 5-cycle warm-up, then 20-cycle calls), against the
same mesh without a communicator. Per call: wall time (launch + exchange + completion) and, with the early
exchange (PAMG_EARLY_XC unset), its start / end against the launch's end. Run it once with and once without
PAMG_EARLY_XC=0 to compare the exchange after the launch."""
import argparse
import os
import sys
import time

import numpy as np
import torch  # noqa: F401

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "p-a_multigrids_amd"))
import pamg  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--calls", type=int, default=40)
ap.add_argument("--parts", type=int, default=2)
a = ap.parse_args()
mesh = pamg.Mesh.strip(32, 16)
mode = "early" if os.environ.get("PAMG_EARLY_XC", "1") != "0" else "after the launch"


def calls(s, diag):
    s.begin_timestep()
    s.vcycle(5)
    s.synchronize()
    out, times = [], []
    for i in range(a.calls):
        if diag:
            s.timing_enable(1 << 15)
            s.timing_reset()
        t0 = time.perf_counter()
        s.vcycle(20)
        s.synchronize()
        out.append((time.perf_counter() - t0) * 1e6)
        if diag:
            t = s.early_exchange_times()
            if t:
                times.append(t)
            s.timing_enable(0)
    return np.array(out), times


plain = pamg.SemiImplicitIterative(mesh, 5, 3, n_smooth=4, solver=3, arith=1)
wp, _ = calls(plain, False)
plain.close()
sp = pamg.SemiImplicitIterative(mesh, 5, 3, n_smooth=4, solver=3, arith=1,
                                self_peer=(pamg.unique_id(), mesh.x_strip_owner(a.parts)))
ws, times = calls(sp, True)
ww, _ = calls(sp, False)
sp.close()
print(f"1,024 un_eles, n_split 5, {a.parts} self-peer parts, exchange {mode}; 20-cycle calls (us, first / median of "
      f"{a.calls}):")
print(f"  no communicator        first {wp[0]:8.1f}  median {np.median(wp):8.1f}")
print(f"  RCCL self-peer (diag)  first {ws[0]:8.1f}  median {np.median(ws):8.1f}")
print(f"  RCCL self-peer         first {ww[0]:8.1f}  median {np.median(ww):8.1f}")
print(f"  charge of the exchange (median, no diag events): {np.median(ww) - np.median(wp):+.1f} us per call")
if times:
    t = np.array(times)
    print(f"  early exchange (median over calls): start {np.median(t[:, 0]):.1f} us, end {np.median(t[:, 1]):.1f} us, "
          f"launch end {np.median(t[:, 2]):.1f} us; exchange ended before the launch in {int((t[:, 1] < t[:, 2]).sum())} "
          f"of {len(t)} calls")
