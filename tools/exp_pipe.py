"""Same-process A/B of the metric pipeline at configs[2]: the three launches
against the persistent one-launch k_pipe (ofhe_hip_plan_pipeline) at several
lags, interleaved rounds, HIP events on the launch stream; every variant's c
must equal the three-launch c.
  EXP_BATCH (1024), EXP_ROUNDS (6), EXP_LAGS ("12h0,12h1,12h2,12h3,6h2,8h2,16h2,12p2h2": lag, optionally w<workgroups per CU>)"""
import os
import re
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
plan = H.NTTPlan(ctx, log_n, qs, rs)
s = torch.cuda.current_stream()
sp = s.cuda_stream
a = torch.empty((B, T, n), dtype=torch.int64, device="cuda")
b = torch.empty_like(a)
c = torch.empty_like(a)
plan.fill_uniform(a.data_ptr(), B, 1, 0, sp)
plan.fill_uniform(b.data_ptr(), B, 2, 0, sp)
plan.ntt_mul_intt(a.data_ptr(), b.data_ptr(), c.data_ptr(), B, sp)
ref = c.clone()
# variants: "three", or "pipe<lag>[w<workgroups per CU>][p<pieces per item>][t][s]"
# (t: static item assignment, h: k_pipe hand-off mode HM)
variants = ["three"] + ["pipe" + x for x in os.environ.get("EXP_LAGS", "12h0,12h1,12h2,12h3,6h2,8h2,16h2,12p2h2").split(",")]
times = {v: [] for v in variants}
for rnd in range(int(os.environ.get("EXP_ROUNDS", "6"))):
    for v in (variants if rnd % 2 == 0 else variants[::-1]):
        if v == "three":
            plan.pipeline(False)
        else:
            m = re.fullmatch(r"(\d+)(?:w(\d+))?(?:p(\d+))?(t?)(?:h(\d))?", v[4:])
            lag, w, pcs, st, hm = m.groups()
            os.environ["OFHE_PIPE_WGS"] = w or ""
            os.environ["OFHE_PIPE_PIECES"] = pcs or "1"
            os.environ["OFHE_PIPE_STATIC"] = "1" if st else "0"
            os.environ["OFHE_PIPE_HM"] = hm or "1"
            plan.pipeline(True, int(lag))
        c.zero_()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        plan.ntt_mul_intt(a.data_ptr(), b.data_ptr(), c.data_ptr(), B, sp)
        e1.record(s)
        e1.synchronize()
        if rnd > 0:
            times[v].append(e0.elapsed_time(e1))
        if not torch.equal(c, ref):
            print("MISMATCH", v, flush=True)
print("faults", plan.pipeline_status(), flush=True)
coeffs = B * T * n
for v in variants:
    med = statistics.median(times[v])
    print(f"{v:8s} {med:8.3f} ms (min {min(times[v]):.3f}) -> {coeffs / med * 1e3:.3e} coeffs/s", flush=True)
