"""CKKS rescale (ofhe_hip_drop_last_and_scale, evaluation form) at configs[4]'s
ring: N = 2^17, 48 -> 47 towers, batch 8; median event time over REPS calls
(for rocprofv3 kernel summaries and A/B runs).  Env: RS_BATCH, RS_REPS, RS_EVAL."""
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "upmem--openfhe_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402
import ofhe_hip as H  # noqa: E402

if os.environ.get("RS_LIB"):  # an A/B variant build (make variant)
    H.LIB_PATH = os.path.join(ROOT, os.environ["RS_LIB"])

log_n, T, B = 17, 48, int(os.environ.get("RS_BATCH", "8"))
ev = os.environ.get("RS_EVAL", "1") == "1"
n = 1 << log_n
q, rq = bench.moduli_chain(log_n, T)
ql = q[-1]
a = [pow(ql, -1, qi) for qi in q[:-1]]
c = [qi - ai for qi, ai in zip(q[:-1], a)]
ctx = H.Context(0)
plan = H.NTTPlan(ctx, log_n, q, rq)
s = torch.cuda.current_stream()
x = torch.empty((B, T, n), dtype=torch.int64, device="cuda")
plan.fill_uniform(x.data_ptr(), B, 8, 0, s.cuda_stream)
out = torch.empty((B, T - 1, n), dtype=torch.int64, device="cuda")
ts = []
for i in range(int(os.environ.get("RS_REPS", "20"))):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    plan.drop_last_and_scale(T, x.data_ptr(), T * n, out.data_ptr(), (T - 1) * n, ev, c, a, B, s.cuda_stream)
    e1.record(s)
    e1.synchronize()
    ts.append(e0.elapsed_time(e1))
med = statistics.median(ts[2:])
print(f"[{os.path.basename(H.LIB_PATH)}] rescale N=2^17 {T}->{T - 1} towers batch {B} eval={ev}: {med:.3f} ms, "
      f"{B * (2 * T - 1) * n * 8 / med / 1e6:.0f} GB/s algorithmic")
