"""Same-process A/B of the metric pipeline's batch chunking at configs[2]
(N = 2^16, 16 towers, batch EXP_BATCH, default 1024): unchunked (the
default) against chunks of C polynomials on one or two streams, with the
intermediates streamed (non-temporal, the default access) or cached
(ofhe_plan_options.cached_intermediates) so a chunk's three launches can meet
in the Infinity Cache.  Interleaved rounds, median ms per call, and every
variant's output compared with the unchunked one.
Env: EXP_BATCH, EXP_ROUNDS (default 6), EXP_CHUNKS (default "8,16,32")."""
import os
import statistics
import sys

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
plans = {"nt": H.NTTPlan(ctx, log_n, qs, rs), "cached": H.NTTPlan(ctx, log_n, qs, rs, cached_intermediates=True)}
s = torch.cuda.current_stream()
sp = s.cuda_stream
a = torch.empty((B, T, n), dtype=torch.int64, device="cuda")
b = torch.empty_like(a)
c = torch.empty_like(a)
plans["nt"].fill_uniform(a.data_ptr(), B, 1, 0, sp)
plans["nt"].fill_uniform(b.data_ptr(), B, 2, 0, sp)
variants = [("unchunked", "nt", 0, 1)]
for cb in (int(x) for x in os.environ.get("EXP_CHUNKS", "8,16,32").split(",")):
    for ns in (1, 2):
        for kind in ("nt", "cached"):
            variants.append((f"chunk{cb}x{ns}-{kind}", kind, cb, ns))
times = {v[0]: [] for v in variants}
ref = None
for rnd in range(int(os.environ.get("EXP_ROUNDS", "6"))):
    for name, kind, cb, ns in (variants if rnd % 2 == 0 else variants[::-1]):
        p = plans[kind]
        p.tune(cb, ns if cb else 1)
        p.ntt_mul_intt(a.data_ptr(), b.data_ptr(), c.data_ptr(), B, sp)  # warm
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(3):
            p.ntt_mul_intt(a.data_ptr(), b.data_ptr(), c.data_ptr(), B, sp)
        e1.record(s)
        e1.synchronize()
        times[name].append(e0.elapsed_time(e1) / 3)
        if rnd == 0:
            h = int(torch.sum(c[:, :, ::97] * 3 + 1).item()) ^ int(torch.sum(c[B // 2]).item())
            if ref is None:
                ref = h
            elif h != ref:
                print("MISMATCH", name, flush=True)
        p.tune(0, 1)
for name, *_ in variants:
    t = times[name]
    print(f"{name:24s} median {statistics.median(t):7.3f} ms  min {min(t):7.3f}  -> "
          f"{B * T * n / statistics.median(t) / 1e6:.3e} coeffs/s", flush=True)
