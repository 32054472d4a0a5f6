"""Runs one stage of the metric pipeline back to back for a fixed time so that
rocm-smi can sample the package power and sclk it settles at (tools/power_probe.sh).
usage: python tools/power_stage.py <stage 0|1|2|all> <seconds> [ENV=VAL ...]  (ENV applied at plan creation)"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "upmem--openfhe_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402
import ofhe_hip as H  # noqa: E402

stage, secs = sys.argv[1], float(sys.argv[2])
for kv in sys.argv[3:]:
    k, v = kv.split("=")
    os.environ[k] = v
B, T, log_n = int(os.environ.get("PS_BATCH", "256")), 16, 16
n = 1 << log_n
qs, rs = bench.moduli_chain(log_n, T)
ctx = H.Context(0)
plan = H.NTTPlan(ctx, log_n, qs, rs)
if os.environ.get("PS_TUNE"):  # "chunk,streams" for the whole pipeline (ofhe_hip_plan_tune)
    cb, ns = (int(x) for x in os.environ["PS_TUNE"].split(","))
    plan.tune(cb, ns)
s = torch.cuda.current_stream()
a = torch.empty((B, T, n), dtype=torch.int64, device="cuda")
b = torch.empty_like(a)
c = torch.empty_like(a)
plan.fill_uniform(a.data_ptr(), B, 1, 0, s.cuda_stream)
plan.fill_uniform(b.data_ptr(), B, 2, 0, s.cuda_stream)
plan.ntt_mul_intt(a.data_ptr(), b.data_ptr(), c.data_ptr(), B, s.cuda_stream)


def run():
    if stage == "all":
        plan.ntt_mul_intt(a.data_ptr(), b.data_ptr(), c.data_ptr(), B, s.cuda_stream)
    else:
        plan.ntt_mul_intt_stage(int(stage), a.data_ptr(), b.data_ptr(), c.data_ptr(), B, s.cuda_stream)


torch.cuda.synchronize()
t0, calls = time.perf_counter(), 0
while time.perf_counter() - t0 < secs:
    for _ in range(20):
        run()
    calls += 20
    torch.cuda.synchronize()
el = time.perf_counter() - t0
print(f"stage {stage} {' '.join(sys.argv[3:])}: {el / calls * 1e3:.3f} ms per call, {calls} calls", flush=True)
