"""Package power while a memory stream runs back to back (tools/power_probe-style
sampling by the caller): torch copies of a buffer that lives in HBM (4 GiB) or
fits the Infinity Cache / L2 (64 MiB, 2 MiB).  usage: python tools/power_mem.py <MiB> <seconds>"""
import sys
import time

import torch

mib, secs = int(sys.argv[1]), float(sys.argv[2])
n = mib * (1 << 20) // 8
a = torch.randint(0, 1 << 60, (n,), dtype=torch.int64, device="cuda")
c = torch.empty_like(a)
c.copy_(a)
torch.cuda.synchronize()
reps = max(1, int(2048 // max(mib, 1)))
t0, k = time.perf_counter(), 0
while time.perf_counter() - t0 < secs:
    for _ in range(reps):
        c.copy_(a)
    k += reps
    torch.cuda.synchronize()
el = time.perf_counter() - t0
print(f"copy {mib} MiB: {2 * n * 8 * k / el / 1e9:.0f} GB/s (read + write)", flush=True)
