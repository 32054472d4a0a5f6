"""Sweep ofhe_hip_plan_tune settings for the metric pipeline (one process, one device).
Prints ms/step per (chunk_batch, streams) and checks outputs are identical."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "upmem--openfhe_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402
import ofhe_hip as H  # noqa: E402

log_n, T, B = 16, 16, int(os.environ.get("EXP_BATCH", "1024"))
n = 1 << log_n
qs, rs = bench.moduli_chain(log_n, T)
ctx = H.Context(0)
plan = H.NTTPlan(ctx, log_n, qs, rs)
g = torch.Generator(device="cuda")
g.manual_seed(1)
a = torch.empty((B, T, n), dtype=torch.int64, device="cuda")
b = torch.empty_like(a)
for t, q in enumerate(qs):
    a[:, t].random_(0, q, generator=g)
    b[:, t].random_(0, q, generator=g)
c = torch.empty_like(a)
ref = None
sp = torch.cuda.current_stream().cuda_stream
settings = [(0, 1), (4, 1), (8, 1), (16, 1), (32, 1), (64, 1), (4, 2), (8, 2), (16, 2), (32, 2), (64, 2), (128, 2)]
for cb, ns in settings:
    plan.tune(cb, ns)
    for _ in range(2):
        plan.ntt_mul_intt(a.data_ptr(), b.data_ptr(), c.data_ptr(), B, sp)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    reps = 8
    for _ in range(reps):
        plan.ntt_mul_intt(a.data_ptr(), b.data_ptr(), c.data_ptr(), B, sp)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / reps * 1e3
    if ref is None:
        ref = c.clone()
        same = True
    else:
        same = bool(torch.equal(ref, c))
    print(f"chunk={cb:4d} streams={ns} ms/step={ms:8.3f} coeffs/s={B*T*n/ms*1e3:.3e} identical={same}", flush=True)
