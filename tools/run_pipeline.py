"""Minimal driver: run the metric pipeline a few times (for rocprofv3 PMC passes).
Env: RUN_LIB (alternate .so path), RUN_BATCH, RUN_REPS, RUN_LOGN (16), RUN_OP
(pipeline | fwd | inv)."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "upmem--openfhe_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402
import ofhe_hip  # noqa: E402

path = os.environ.get("RUN_LIB", ofhe_hip.LIB_PATH)
L = ctypes.CDLL(path)
for name, (res, args) in ofhe_hip._SIGS.items():
    if hasattr(L, name):
        getattr(L, name).restype, getattr(L, name).argtypes = res, args
vp = ctypes.c_void_p
log_n, T, B = int(os.environ.get("RUN_LOGN", "16")), 16, int(os.environ.get("RUN_BATCH", "256"))
op = os.environ.get("RUN_OP", "pipeline")
n = 1 << log_n
qs, rs = bench.moduli_chain(log_n, T)
arr = lambda v: (ctypes.c_uint64 * len(v))(*v)  # noqa: E731
ctx, plan = vp(), vp()
assert L.ofhe_hip_init(0, ctypes.byref(ctx)) == 0
assert L.ofhe_hip_plan_create(ctx, log_n, T, arr(qs), arr(rs), ctypes.byref(plan)) == 0
a = torch.randint(0, 2**59, (B, T, n), dtype=torch.int64, device="cuda")
b = torch.randint(0, 2**59, (B, T, n), dtype=torch.int64, device="cuda")
c = torch.empty_like(a)
sp = vp(torch.cuda.current_stream().cuda_stream)
for t, q in enumerate(qs):  # canonical inputs (the forward transform's contract)
    a[:, t] %= q
    b[:, t] %= q
for _ in range(int(os.environ.get("RUN_REPS", "3"))):
    if op == "fwd":
        assert L.ofhe_hip_ntt_fwd(plan, vp(a.data_ptr()), B, sp) == 0
    elif op == "inv":
        assert L.ofhe_hip_ntt_inv(plan, vp(b.data_ptr()), B, sp) == 0
    else:
        assert L.ofhe_hip_ntt_mul_intt(plan, vp(a.data_ptr()), vp(b.data_ptr()), vp(c.data_ptr()), B, sp) == 0
torch.cuda.synchronize()
print("done", path)
