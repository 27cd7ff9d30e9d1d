"""50 pipelined V-cycles with no HIP-event timing (for rocprofv3 --kernel-trace: the
gaps between consecutive launches). Arg: partitions N (rank 0's x-strip, detached)."""
import os
import sys

import torch  # noqa: F401

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "p-a_multigrids_amd"))
import pamg  # noqa: E402

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
mesh = pamg.Mesh.read(os.path.join(ROOT, "tests", "meshes", "untitled8192.msh"))
N = int(sys.argv[1]) if len(sys.argv) > 1 else 1
comm = None if N == 1 else (N, 0, None, mesh.x_strip_owner(N))
s = pamg.SemiImplicitIterative(mesh, 5, 3, n_smooth=4, solver=3, arith=1, comm=comm)
s.begin_timestep()
s.vcycle(5)
s.synchronize()
s.vcycle(50)
s.synchronize()
