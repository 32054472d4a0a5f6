"""A/B timing of compile-time variants (upmem--openfhe_amd/lib/variants/*.so)
on the configs[4] key switch (N = 2^17, Q = 48, P = 16, dnum = 3), in ONE
process, interleaved rounds; checks every variant's output equals the first's.
Env: EXP_KS_BATCH (default 8), EXP_ROUNDS (default 5), EXP_ONLY, EXP_TOGGLE."""
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
log_n, sq, sp, dnum = 17, 48, 16, 3
n = 1 << log_n
B = int(os.environ.get("EXP_KS_BATCH", "8"))
allq, allr = bench.moduli_chain(log_n, sq + sp)
arr = lambda v: (ctypes.c_uint64 * len(v))(*v)  # noqa: E731
g = torch.Generator(device="cuda")
g.manual_seed(5)


def uniform(shape, moduli):
    x = torch.empty(shape, dtype=torch.int64, device="cuda")
    for t, m in enumerate(moduli):
        x[..., t, :].random_(0, m, generator=g)
    return x


c = uniform((B, sq, n), allq[:sq])
kb = uniform((dnum, sq + sp, n), allq)
ka = uniform((dnum, sq + sp, n), allq)
o0 = torch.empty((B, sq, n), dtype=torch.int64, device="cuda")
o1 = torch.empty_like(o0)
libs = []
for p in paths:
    L = ctypes.CDLL(p)
    for name, (res, args) in ofhe_hip._SIGS.items():
        if hasattr(L, name):
            getattr(L, name).restype, getattr(L, name).argtypes = res, args
    ctx = vp()
    assert L.ofhe_hip_init(0, ctypes.byref(ctx)) == 0
    # EXP_TOGGLE="field=v;field2=v": one more engine per entry, created with
    # those ofhe_ks_options fields set (ofhe_hip.KsOptions: separate_cols,
    # separate_icol, chunk, single_stream, plan.split, plan.generic_moduli),
    # timed in the same interleaved rounds
    toggle = os.environ.get("EXP_TOGGLE")
    for tv in [None] + (toggle.split(";") if toggle else []):
        opt = ofhe_hip.KsOptions()
        for kv in filter(None, (tv or "").split(",")):
            k, _, v = kv.partition("=")
            obj, fld = (opt.plan, k[5:]) if k.startswith("plan.") else (opt, k)
            setattr(obj, fld, int(v or "1"))
        ks = vp()
        assert L.ofhe_hip_ks_create_ex(ctx, log_n, sq, arr(allq[:sq]), arr(allr[:sq]), sp, arr(allq[sq:]),
                                       arr(allr[sq:]), dnum, ofhe_hip._opt_ptr(opt), ctypes.byref(ks)) == 0, \
            L.ofhe_hip_last_error()
        libs.append((os.path.basename(p) + (f"+{tv}" if tv else ""), L, ks))
s = torch.cuda.current_stream()
spt = vp(s.cuda_stream)
times = {nm: [] for nm, _, _ in libs}
ref = None
for rnd in range(int(os.environ.get("EXP_ROUNDS", "5"))):
    # alternate the order every round: the engine timed first in a round
    # measured ~2-3 % faster whichever it was
    for nm, L, ks in (libs if rnd % 2 == 0 else libs[::-1]):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        assert L.ofhe_hip_ks_core(ks, sq, vp(c.data_ptr()), vp(kb.data_ptr()), vp(ka.data_ptr()), vp(o0.data_ptr()),
                                  vp(o1.data_ptr()), 0, B, spt) == 0
        e1.record(s)
        e1.synchronize()
        if rnd > 0:
            times[nm].append(e0.elapsed_time(e1))
        out = torch.cat([o0, o1])
        if ref is None:
            ref = out.clone()
        elif not torch.equal(ref, out):
            print("MISMATCH", nm, flush=True)
for nm, tt in times.items():
    med = statistics.median(tt)
    print(f"{nm:40s} ks_core {med:7.3f} ms ({B} ciphertexts) -> {B / med * 1e3:.1f} keyswitch/s "
          f"[min {min(tt):.3f} max {max(tt):.3f}; by round: {' '.join(f'{x:.2f}' for x in tt)}]", flush=True)
