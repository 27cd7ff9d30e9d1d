"""Round 6 debug: the agglomerated coarsest level on a local group (prints every rank's progress)."""
import faulthandler
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "p-a_multigrids_amd"))
os.environ.setdefault("PAMG_COMM_TIMEOUT_S", "20")
import pamg  # noqa: E402
from pamg.solver import local_group, run_ranks  # noqa: E402

faulthandler.dump_traceback_later(45, exit=False)
mesh_name, S, L, parts, cycle = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5])
m = pamg.Mesh.read(os.path.join(ROOT, "tests", "meshes", mesh_name))
owner = m.x_strip_owner(parts)
t0 = time.time()


def say(*a):
    print(f"[{time.time() - t0:7.2f} {threading.current_thread().name}]", *a, flush=True)


ps = [pamg.SemiImplicitIterative(m, S, L, solver=3, cycle=cycle, op=1, comm=(parts, r, None, owner)) for r in range(parts)]
say("handles made")
local_group(ps)
say("group bound")


def drive(p):
    for step in range(2):
        say("begin_timestep", step)
        p.begin_timestep()
        say("vcycle(2)")
        p.vcycle(2)
        say("vcycle done")
    p.synchronize()
    say("synced")


run_ranks(ps, drive)
say("all done")
full = pamg.SemiImplicitIterative(m, S, L, solver=3, cycle=cycle, op=1)
for _ in range(2):
    full.begin_timestep()
    full.vcycle(2)
import numpy as np  # noqa: E402
ref = full.state()
for r, p in enumerate(ps):
    own = np.flatnonzero(owner == r)
    for k, v in p.state().items():
        same = np.array_equal(v, ref[k][:, :, own])
        if not same:
            say(f"rank {r} {k} differs: max {np.abs(v - ref[k][:, :, own]).max():.3e}")
say("compared")
faulthandler.cancel_dump_traceback_later()
