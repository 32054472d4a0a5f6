"""Block pass of the metric pipeline with the batch split between k_block
(VALU butterflies) and k_block_m16 (matrix cores, waits on MFMA latency) on two
streams at once, against either alone: whether the butterfly waves fill the
matrix-core waves' idle issue slots under the package power cap.  One process;
outputs of the split run checked against k_block's.  Env: EXP_BATCH (512)."""
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "upmem--openfhe_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402
import ofhe_hip as H  # noqa: E402

log_n, T, B = 16, 16, int(os.environ.get("EXP_BATCH", "512"))
n = 1 << log_n
W = T * n
qs, rs = bench.moduli_chain(log_n, T)
ctx = H.Context(0)
pk = H.NTTPlan(ctx, log_n, qs, rs)
os.environ["OFHE_BLOCK_M16"] = "1"
pm = H.NTTPlan(ctx, log_n, qs, rs)
del os.environ["OFHE_BLOCK_M16"]
s0 = torch.cuda.current_stream()
s1 = torch.cuda.Stream()
a = torch.empty((B, T, n), dtype=torch.int64, device="cuda")
b = torch.empty_like(a)
pk.fill_uniform(a.data_ptr(), B, 1, 0, s0.cuda_stream)
pk.fill_uniform(b.data_ptr(), B, 2, 0, s0.cuda_stream)
c0 = torch.empty_like(a)
pk.ntt_mul_intt_stage(0, a.data_ptr(), b.data_ptr(), c0.data_ptr(), B, s0.cuda_stream)
mid = c0.clone()


def run(kind, f):
    """kind: 'k', 'm' or 'mix' (fraction f of the batch on the m16 plan)."""
    c0.copy_(mid)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    ev0.record(s0)
    if kind == "k":
        pk.ntt_mul_intt_stage(1, a.data_ptr(), b.data_ptr(), c0.data_ptr(), B, s0.cuda_stream)
    elif kind == "m":
        pm.ntt_mul_intt_stage(1, a.data_ptr(), b.data_ptr(), c0.data_ptr(), B, s0.cuda_stream)
    else:
        bm = max(1, int(round(B * f)))
        bk = B - bm
        s1.wait_event(ev0)
        pk.ntt_mul_intt_stage(1, a.data_ptr(), b.data_ptr(), c0.data_ptr(), bk, s0.cuda_stream)
        off = bk * W * 8
        pm.ntt_mul_intt_stage(1, a.data_ptr() + off, b.data_ptr() + off, c0.data_ptr() + off, bm, s1.cuda_stream)
        e = torch.cuda.Event()
        e.record(s1)
        s0.wait_event(e)
    ev1.record(s0)
    ev1.synchronize()
    return ev0.elapsed_time(ev1)


run("k", 0)
cfgs = [("k_block", "k", 0), ("m16", "m", 0)] + [(f"mix m16 {f:.2f}", "mix", f) for f in (0.2, 0.33, 0.5)]
times = {nm: [] for nm, *_ in cfgs}
for rnd in range(int(os.environ.get("EXP_ROUNDS", "6"))):
    for nm, kind, f in (cfgs if rnd % 2 == 0 else cfgs[::-1]):
        times[nm].append(run(kind, f))
for nm in times:
    ms = statistics.median(times[nm][1:])
    print(f"{nm:16s} block pass {ms:7.3f} ms  ({B * W / ms * 1e3:.3e} coeffs/s)  all {', '.join(f'{t:.3f}' for t in times[nm])}",
          flush=True)
