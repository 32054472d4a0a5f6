"""Standalone timing of ApproxSwitchCRTBasis (ofhe_hip_approx_switch_crt_basis)
at the key switch's shape: N = 2^17, 16 source towers -> 48 target towers
(ModUp of one digit, and ModDown's P -> Q), batch EXP_BATCH (default 8), one
stream, nothing else running.  EXP_LIB times a variant build.  Prints one JSON
object: ms per call and the HBM rate on (16 + 48) * 8 B per coefficient."""
import json
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "upmem--openfhe_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402
import ofhe_hip as H  # noqa: E402

if os.environ.get("EXP_LIB"):
    H.LIB_PATH = os.environ["EXP_LIB"]

log_n, sq, sp = 17, 16, 48
B = int(os.environ.get("EXP_BATCH", "8"))
n = 1 << log_n
allq, _ = bench.moduli_chain(log_n, sq + sp)
q, p = allq[:sq], allq[sq:]
Q = math.prod(q)
qhat = [Q // qi for qi in q]
qhinv = [pow(h % qi, -1, qi) for h, qi in zip(qhat, q)]
qhmodp = [h % pj for h in qhat for pj in p]
ctx = H.Context(0)
bc = H.BaseConverter(ctx, log_n, q, p, qhinv, qhmodp)
s = torch.cuda.current_stream()
x = torch.empty((B, sq, n), dtype=torch.int64, device="cuda")
for t, qt in enumerate(q):
    x[:, t, :].random_(0, qt)
out = torch.empty((B, sp, n), dtype=torch.int64, device="cuda")
res = {"config": f"N=2^{log_n}, {sq} -> {sp} towers, batch {B}", "lib": H.LIB_PATH}
bc.switch(x.data_ptr(), out.data_ptr(), B, s.cuda_stream)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
reps = 20
e0.record(s)
for _ in range(reps):
    bc.switch(x.data_ptr(), out.data_ptr(), B, s.cuda_stream)
e1.record(s)
e1.synchronize()
ms = e0.elapsed_time(e1) / reps
coeffs = B * n
res.update({"ms": ms, "gbs": coeffs * (sq + sp) * 8 / (ms * 1e-3) / 1e9,
            "checksum": int(out.sum().item())})
print(json.dumps(res))
