"""The one-launch-per-cycle form (call schedule 1) on bench.py's workload alone, for rocprofv3
PMC passes of its pipelined launch (profiles/pmc_vcycle_pipe.json; GPU box only)."""
import os
import sys

import torch  # noqa: F401

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "p-a_multigrids_amd"))
import pamg  # noqa: E402

mesh = pamg.Mesh.read(os.path.join(ROOT, "tests", "meshes", "untitled8192.msh"))
s = pamg.SemiImplicitIterative(mesh, 5, 3, n_smooth=4, solver=3, arith=1, fused=3)
s.set_call_schedule(1)
s.begin_timestep()
s.vcycle(int(sys.argv[1]) if len(sys.argv) > 1 else 20)
s.synchronize()
s.close()
print("ok")
