"""Phase timeline of the face operator's two-sweep passes (k_face_pp) on bench.py's mesh (GPU box only):
runs scripts/face_probe.py's workload with a PAMG_STAMPS=1 build (PAMG_LIB) and PAMG_PP_STAMPS, then reads the
per-workgroup stamps (start, loads done, ghost update done, sweep 1 done, sweep 2 done, stores drained) of the
level-1 launches and prints the median phase durations, a workgroup's life against the launch's span, and how
the workgroups' starts bunch into rounds."""
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
lib = os.path.join(ROOT, "scripts", "ablibs", "pp_stamps.so")
path = os.path.join(tempfile.mkdtemp(), "pp.bin")
env = dict(os.environ, PAMG_LIB=lib, PAMG_PP_STAMPS=path)
r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "face_probe.py"), "5", "0"], env=env,
                   capture_output=True, text=True, timeout=300)
print(r.stdout.splitlines()[0] if r.stdout else r.stderr[-2000:])
raw = np.fromfile(path, dtype=np.int64)
launches = []
i = 0
while i < len(raw):
    g, ns, nsub, K = raw[i:i + 4]
    st = raw[i + 4:i + 4 + g * ns].reshape(g, ns)
    i += 4 + g * ns
    launches.append((int(nsub), int(K), st))
names = ["loads", "ghost", "sweep 1", "sweep 2", "stores"]
for nsub in (1024, 256):
    sel = [st for n, K, st in launches if n == nsub and K == 2][-10:]
    if not sel:
        continue
    d = np.concatenate([np.diff(st, axis=1) for st in sel]) * 10e-3   # us
    life = np.concatenate([(st[:, -1] - st[:, 0]) for st in sel]) * 10e-3
    span = np.array([(st[:, -1].max() - st[:, 0].min()) * 10e-3 for st in sel])
    print(f"k_face_pp<{nsub}, .., K=2>: {len(sel)} launches of {sel[0].shape[0]} workgroups; launch span median "
          f"{np.median(span):.1f} us; workgroup life median {np.median(life):.2f} us")
    print("   phase medians (us): " + ", ".join(f"{n} {np.median(d[:, k]):.2f}" for k, n in enumerate(names)))
    st = sel[-1]
    t0 = st[:, 0].min()
    starts = np.sort((st[:, 0] - t0) * 10e-3)
    hist, edges = np.histogram(starts, bins=24)
    print("   workgroup starts over the last launch (us -> count): " +
          " ".join(f"{edges[k]:.0f}:{hist[k]}" for k in range(len(hist))))
