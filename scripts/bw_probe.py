"""HBM bandwidth reference points on the box (torch's own kernels), to read the
fused V-cycle's GB/s against: read-only, copy (1R1W), add (2R1W)."""
import time

import torch

n = 1 << 27  # 1 GiB of fp64
a = torch.rand(n, dtype=torch.float64, device="cuda")
b = torch.rand(n, dtype=torch.float64, device="cuda")
c = torch.empty_like(a)


def bench(f, nbytes, reps=20):
    f()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        f()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / reps
    return nbytes / dt / 1e12


print("read (sum)  TB/s", round(bench(lambda: a.sum(), 8 * n), 2))
print("copy 1R1W   TB/s", round(bench(lambda: c.copy_(a), 16 * n), 2))
print("add  2R1W   TB/s", round(bench(lambda: torch.add(a, b, out=c), 24 * n), 2))
print("fill 0R1W   TB/s", round(bench(lambda: c.fill_(1.0), 8 * n), 2))
