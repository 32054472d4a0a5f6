"""Chunked metric pipeline with the intermediates in a reused chunk-sized
scratch (OFHE_CHUNK_SCRATCH at plan creation) against the unchunked pipeline
and the chunks-through-c form, one process, rounds interleaved; outputs checked
identical.  Env: EXP_BATCH (1024), EXP_ROUNDS (4)."""
import os
import statistics
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
plain = H.NTTPlan(ctx, log_n, qs, rs)
os.environ["OFHE_CHUNK_SCRATCH"] = "1"
scr = H.NTTPlan(ctx, log_n, qs, rs)
del os.environ["OFHE_CHUNK_SCRATCH"]
sp = torch.cuda.current_stream().cuda_stream
a = torch.empty((B, T, n), dtype=torch.int64, device="cuda")
b = torch.empty_like(a)
plain.fill_uniform(a.data_ptr(), B, 1, 0, sp)
plain.fill_uniform(b.data_ptr(), B, 2, 0, sp)
c = torch.empty_like(a)
cfgs = [("unchunked", plain, 0, 1)]
for cb in [int(x) for x in os.environ.get("EXP_CHUNKS", "8,16,32,64").split(",")]:
    for ns in (1, 2):
        cfgs.append((f"scratch cb={cb} s={ns}", scr, cb, ns))
        cfgs.append((f"via-c   cb={cb} s={ns}", plain, cb, ns))
times = {nm: [] for nm, *_ in cfgs}
ref = None
for rnd in range(int(os.environ.get("EXP_ROUNDS", "4"))):
    for nm, pl, cb, ns in (cfgs if rnd % 2 == 0 else cfgs[::-1]):
        pl.tune(cb, ns)
        pl.ntt_mul_intt(a.data_ptr(), b.data_ptr(), c.data_ptr(), B, sp)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(5):
            pl.ntt_mul_intt(a.data_ptr(), b.data_ptr(), c.data_ptr(), B, sp)
        torch.cuda.synchronize()
        times[nm].append((time.perf_counter() - t0) / 5 * 1e3)
        if ref is None:
            ref = c.clone()
        elif not torch.equal(ref, c):
            print("MISMATCH", nm, flush=True)
    print("round", rnd, "done", flush=True)
for nm in times:
    ms = statistics.median(times[nm])
    print(f"{nm:24s} {ms:8.3f} ms/step  {B * T * n / ms * 1e3:.3e} coeffs/s  (all {', '.join(f'{t:.2f}' for t in times[nm])})",
          flush=True)
