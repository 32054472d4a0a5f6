"""A/B timing of compile-time kernel variants (upmem--openfhe_amd/lib/variants/*.so)
in ONE process on one device, interleaved rounds (cdna_hip_programming.md §5.4 rule 24).
Times each pipeline stage with HIP events on the launch stream and checks every
variant's output equals the first variant's."""
import ctypes
import glob
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "upmem--openfhe_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402
import ofhe_hip  # noqa: E402

vp = ctypes.c_void_p
paths = sorted(glob.glob(os.path.join(ROOT, "upmem--openfhe_amd", "lib", "variants", "*.so")))
only = os.environ.get("EXP_ONLY")
if only:
    paths = [p for p in paths if any(o in os.path.basename(p) for o in only.split(","))]
log_n, T, B = int(os.environ.get("EXP_LOGN", "16")), 16, int(os.environ.get("EXP_BATCH", "256"))
n = 1 << log_n
qs, rs = bench.moduli_chain(log_n, T)
arr = lambda v: (ctypes.c_uint64 * len(v))(*v)  # noqa: E731
libs = []
# EXP_CONFIGS: ';'-separated plan options (ofhe_hip.PlanOptions fields), e.g.
# ";split=1;generic_moduli=1" -- one engine per entry and library
configs = os.environ.get("EXP_CONFIGS", "").split(";")
for p in paths:
    L = ctypes.CDLL(p)
    for name, (res, args) in ofhe_hip._SIGS.items():
        if hasattr(L, name):
            f = getattr(L, name)
            f.restype, f.argtypes = res, args
    ctx = vp()
    assert L.ofhe_hip_init(0, ctypes.byref(ctx)) == 0
    for cfg in configs:
        opt = ofhe_hip.PlanOptions()
        for kv in filter(None, cfg.split(",")):
            k, v = kv.split("=")
            setattr(opt, k, int(v))
        plan = vp()
        assert L.ofhe_hip_plan_create_ex(ctx, log_n, T, arr(qs), arr(rs), ofhe_hip._opt_ptr(opt),
                                         ctypes.byref(plan)) == 0, L.ofhe_hip_last_error()
        libs.append((os.path.basename(p) + ("[" + cfg + "]" if cfg else ""), L, plan))

g = torch.Generator(device="cuda")
g.manual_seed(3)
a = torch.empty((B, T, n), dtype=torch.int64, device="cuda")
b = torch.empty_like(a)
for t, q in enumerate(qs):
    a[:, t].random_(0, q, generator=g)
    b[:, t].random_(0, q, generator=g)
c = torch.empty_like(a)
s = torch.cuda.current_stream()
sp = vp(s.cuda_stream)
times = {nm: {0: [], 1: [], 2: [], "all": [], "fwd": [], "inv": []} for nm, _, _ in libs}
ref = None
ref_t = {}
for rnd in range(int(os.environ.get("EXP_ROUNDS", "6"))):
    # alternate the order every round (the first engine of a round has an edge)
    for nm, L, plan in (libs if rnd % 2 == 0 else libs[::-1]):
        for st in (0, 1, 2, "all"):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            if st == 0 or st == "all":
                pre = []
            else:
                pre = [0] if st == 1 else [0, 1]
            for p_ in pre:
                L.ofhe_hip_ntt_mul_intt_stage(plan, p_, vp(a.data_ptr()), vp(b.data_ptr()), vp(c.data_ptr()), B, sp)
            e0.record(s)
            if st == "all":
                rc = L.ofhe_hip_ntt_mul_intt(plan, vp(a.data_ptr()), vp(b.data_ptr()), vp(c.data_ptr()), B, sp)
            else:
                rc = L.ofhe_hip_ntt_mul_intt_stage(plan, st, vp(a.data_ptr()), vp(b.data_ptr()), vp(c.data_ptr()), B, sp)
            assert rc == 0
            e1.record(s)
            e1.synchronize()
            if rnd > 0:
                times[nm][st].append(e0.elapsed_time(e1))
        # standalone forward / inverse transforms (FWD / INV block modes)
        for st in ("fwd", "inv"):
            x = a.clone()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            fn = L.ofhe_hip_ntt_fwd if st == "fwd" else L.ofhe_hip_ntt_inv
            assert fn(plan, vp(x.data_ptr()), B, sp) == 0
            e1.record(s)
            e1.synchronize()
            if rnd > 0:
                times[nm][st].append(e0.elapsed_time(e1))
            if st not in ref_t:
                ref_t[st] = x
            elif not torch.equal(ref_t[st], x):
                print("MISMATCH", nm, st, flush=True)
        if ref is None:
            ref = c.clone()
        elif not torch.equal(ref, c):
            print("MISMATCH", nm, flush=True)
coeffs = B * T * n
for nm in times:
    tt = times[nm]
    med = {k: statistics.median(v) for k, v in tt.items()}
    print(f"{nm:44s} cols_f {med[0]:7.3f} block {med[1]:7.3f} cols_i {med[2]:7.3f} all {med['all']:7.3f} ms "
          f"-> {coeffs / med['all'] * 1e3:.3e} coeffs/s (min all {min(tt['all']):.3f}) "
          f"| ntt fwd {med['fwd']:7.3f} inv {med['inv']:7.3f} ms", flush=True)
