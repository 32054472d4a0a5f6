"""HBM bandwidth of the element-wise kernels (ModMul / ModAdd / ModSub vector x
vector: 24 B per coefficient; scalar ops: 16 B) and of the standalone
transforms (16 B per coefficient, two passes) at N = 2^16, 16 towers, batch
EXP_BATCH (default 256).  Prints one JSON object."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "upmem--openfhe_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402
import ofhe_hip as H  # noqa: E402

if os.environ.get("EXP_LIB"):  # A/B: time a variant build (upmem--openfhe_amd/lib/variants)
    H.LIB_PATH = os.environ["EXP_LIB"]

log_n, T, B = 16, 16, int(os.environ.get("EXP_BATCH", "256"))
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
coeffs = B * T * n
sc = [q // 3 for q in qs]
ops = {
    "modmul_vv": (lambda: plan.mod_mul(a.data_ptr(), b.data_ptr(), c.data_ptr(), B, sp), 24),
    "modadd_vv": (lambda: plan.mod_add(a.data_ptr(), b.data_ptr(), c.data_ptr(), B, sp), 24),
    "modsub_vv": (lambda: plan.mod_sub(a.data_ptr(), b.data_ptr(), c.data_ptr(), B, sp), 24),
    "modmul_scalar": (lambda: plan.mod_mul_scalar(a.data_ptr(), sc, c.data_ptr(), B, sp), 16),
    "modadd_scalar": (lambda: plan.mod_add_scalar(a.data_ptr(), sc, c.data_ptr(), B, sp), 16),
    "ntt_fwd": (lambda: plan.forward(c.data_ptr(), B, sp), 32),
    "ntt_inv": (lambda: plan.inverse(c.data_ptr(), B, sp), 32),
    # torch's own streaming kernels on the same buffers: the achievable rate
    "torch_copy": (lambda: c.copy_(a), 16),
    "torch_add": (lambda: torch.add(a, b, out=c), 24),
}
out = {"config": f"N=2^{log_n}, towers={T}, batch={B}", "lib": H.LIB_PATH, "kernels": {}}
for name, (fn, bpc) in ops.items():
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(10):
        fn()
    e1.record(s)
    e1.synchronize()
    ms = e0.elapsed_time(e1) / 10
    out["kernels"][name] = {"ms": ms, "bytes_per_coeff": bpc, "gbs": coeffs * bpc / (ms * 1e-3) / 1e9,
                            "hbm_frac": coeffs * bpc / (ms * 1e-3) / 8e12}
print(json.dumps(out, indent=1))
