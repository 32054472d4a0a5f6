#!/usr/bin/env python3
"""Headline benchmark: 64-bit coefficients/s for c = INTT(NTT(a) (.) b) on
N = 2^16, 16 towers, batch 1024 per GPU (BASELINE.json configs[2]), with the
dominant kernel's HBM-roofline fraction and a CPU baseline on the host cores.

Single GPU:   python bench.py [--steps K --warmup W]
N GPUs:       python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \
                  --master-port P bench.py --gpus N
Each rank processes its own batch shard (weak scaling: per-GPU work fixed, no
collective on the data path).  RCCL is used once at setup to broadcast a
synthetic evaluation key from rank 0 (the only exchange the north star names).

Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import socket
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "upmem--openfhe_amd"))

METRIC = "64-bit coeffs/sec for NTT+Hadamard+INTT, N=2^16, 16 towers; % HBM roofline"
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: 8 TB/s spec
ALG_BYTES_PER_COEFF = 24       # read a, read b, write c
STAGE_NAMES = {0: "colpass<fwd>", 1: "k_block<fused>", 2: "colpass<inv>"}  # colpass = k_tcols (N=2^16) or k_cols


def moduli_chain(log_n, towers, bits=60):
    """poly-benchmark modulus chain (benchmark/src/poly-benchmark-16k.cpp:89-96)
    and minimal primitive 2N-th roots (nbtheory-impl.h:183-231).  Product-side
    setup code (not the oracle): deterministic Miller-Rabin in Python ints."""
    m = 2 << log_n

    def is_prime(n):
        if n < 2:
            return False
        for p in (2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37):
            if n % p == 0:
                return n == p
        d, s = n - 1, 0
        while d % 2 == 0:
            d //= 2
            s += 1
        for a in (2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37):
            x = pow(a, d, n)
            if x in (1, n - 1):
                continue
            for _ in range(s - 1):
                x = x * x % n
                if x == n - 1:
                    break
            else:
                return False
        return True

    q = (1 << bits) + 1
    while not is_prime(q):
        q += m
    qs, roots = [], []
    for _ in range(towers):
        q -= m
        while not is_prime(q):
            q -= m
        qs.append(q)
        e = (q - 1) // m
        c = 2
        while True:
            x = pow(c, e, q)
            if pow(x, m // 2, q) == q - 1:
                break
            c += 1
        x2 = x * x % q
        best, y = x, x
        for _ in range(m // 2 - 1):
            y = y * x2 % q
            if y < best:
                best = y
        roots.append(best)
    return qs, roots


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--log-n", type=int, default=16)
    ap.add_argument("--towers", type=int, default=16)
    ap.add_argument("--batch", type=int, default=1024, help="polynomials per GPU")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline budget (0 = skip)")
    ap.add_argument("--no-check", action="store_true")
    ap.add_argument("--workload", default="pipeline", choices=["pipeline", "keyswitch"],
                    help="pipeline = the headline metric (configs[2]); keyswitch = configs[4] HYBRID "
                         "key switching (secondary line, not the headline)")
    ap.add_argument("--shard", default="batch", choices=["batch", "towers"],
                    help="batch = every rank runs its own batch of --batch (weak scaling, the default line); "
                         "towers = configs[3]: --towers split across ranks, same batch on each (strong scaling)")
    ap.add_argument("--ks-batch", type=int, default=8, help="ciphertext polynomials per GPU (keyswitch)")
    ap.add_argument("--pcie-batch", type=int, default=32, help="polynomials per chunk of the PCIe-inclusive run")
    ap.add_argument("--pcie-chunks", type=int, default=16, help="chunks of the PCIe-inclusive run (0 = skip)")
    args = ap.parse_args()
    if args.workload == "keyswitch":
        return bench_keyswitch(args)

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    import ofhe_hip as H
    import shard

    log_n, T_total, B = args.log_n, args.towers, args.batch
    if args.shard == "batch":
        # weak scaling: every rank owns a batch shard of the same size
        _, B_rank = shard.shard_batch(args.batch * world, rank, world)
        assert B_rank == args.batch
        t_start, T = 0, T_total
    else:
        # strong scaling (configs[3]): a contiguous tower range per rank
        t_start, T = shard.shard_towers(T_total, rank, world)
        if T == 0:
            raise SystemExit(f"--shard towers needs at least one tower per rank ({T_total} over {world})")

    ctx = H.Context(local)
    n = 1 << log_n
    qs_all, roots_all = moduli_chain(log_n, T_total)
    qs, roots = qs_all[t_start:t_start + T], roots_all[t_start:t_start + T]
    plan = H.NTTPlan(ctx, log_n, qs, roots)

    # synthetic inputs, uniform residues mod q_t, generated on the device
    g = torch.Generator(device=dev)
    g.manual_seed(0x5EED + rank)
    a = torch.empty((B, T, n), dtype=torch.int64, device=dev)
    b = torch.empty((B, T, n), dtype=torch.int64, device=dev)
    for t, q in enumerate(qs):
        a[:, t, :].random_(0, q, generator=g)
        b[:, t, :].random_(0, q, generator=g)
    c = torch.empty_like(a)
    stream = torch.cuda.current_stream(dev)
    sp = stream.cuda_stream

    # RCCL broadcast of a synthetic hybrid key-switching key (configs[3]; setup,
    # outside the timed loop -- the only collective the path has)
    bcast, comm = None, None
    if world > 1:
        key = torch.empty(shard.evalkey_words(T_total, log_n, 3), dtype=torch.int64, device=dev)
        if rank == 0:
            key.random_(0, qs[-1], generator=g)
        bfn, backend, comm = shard.key_broadcaster(ctx, rank, world)
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        bfn(key, 0)
        torch.cuda.synchronize()
        bcast = {"bytes": key.numel() * 8, "ms": (time.perf_counter() - t0) * 1e3, "backend": backend,
                 "verified": shard.same_on_all_ranks(key)}
        del key

    def step():
        plan.ntt_mul_intt(a.data_ptr(), b.data_ptr(), c.data_ptr(), B, sp)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        elapsed = shard.max_over_ranks(elapsed, device=dev)
    coeffs_per_step = B * T * n * world if args.shard == "batch" else B * T_total * n
    value = coeffs_per_step * args.steps / elapsed
    ms_per_step = elapsed / args.steps * 1e3

    # per-kernel durations with HIP events on the launch stream (separate pass)
    kernels = {}
    reps = max(3, min(args.steps, 10))
    for st in (0, 1, 2):
        if log_n <= 12 and st != 1:
            continue
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        plan.ntt_mul_intt_stage(0, a.data_ptr(), b.data_ptr(), c.data_ptr(), B, sp)
        plan.ntt_mul_intt_stage(1, a.data_ptr(), b.data_ptr(), c.data_ptr(), B, sp)
        ev0.record(stream)
        for _ in range(reps):
            plan.ntt_mul_intt_stage(st, a.data_ptr(), b.data_ptr(), c.data_ptr(), B, sp)
        ev1.record(stream)
        ev1.synchronize()
        kernels[STAGE_NAMES[st]] = ev0.elapsed_time(ev1) / reps
    dominant = max(kernels, key=kernels.get)
    kms = kernels[dominant]
    coeffs_rank = B * T * n
    achieved = ALG_BYTES_PER_COEFF * coeffs_rank / (kms * 1e-3) / 1e9
    traffic = None
    pmc_path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(pmc_path):
        try:
            pm = json.load(open(pmc_path))
            ent = pm.get("kernels", {}).get(dominant)
            if ent and ent.get("batch") == B and ent.get("log_n") == log_n and ent.get("towers") == T:
                traffic = ent.get("hbm_bytes_per_launch")
        except Exception:
            traffic = None

    # VALU issue rate of the dominant kernel from the SQ counters
    # (tools/pmc_valu.sh -> profiles/pmc_valu.json): the path is bound by
    # integer-VALU issue, not HBM
    valu = None
    vpath = os.path.join(ROOT, "profiles", "pmc_valu.json")
    if os.path.exists(vpath):
        try:
            valu = json.load(open(vpath)).get("kernels", {}).get(dominant)
        except Exception:
            valu = None

    # spot parity check against the oracle (one tower of two batch entries)
    parity = None
    if not args.no_check and rank == 0:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import numpy as np
        import oracle as O

        step()
        torch.cuda.synchronize()
        ok = True
        for bi, ti in ((0, 0), (B - 1, T - 1)):
            tb = O.Tables(n, [qs[ti]], [roots[ti]])
            aa = a[bi, ti].cpu().numpy().view(np.uint64).reshape(1, 1, n)
            bb = b[bi, ti].cpu().numpy().view(np.uint64).reshape(1, 1, n)
            cc = c[bi, ti].cpu().numpy().view(np.uint64).reshape(1, 1, n)
            ok = ok and bool(np.array_equal(cc, O.ntt_mul_intt(aa, bb, tb)))
        parity = ok

    # PCIe-inclusive rate (DESIGN.md §(d)): a and b in pinned host memory, c back
    # to host, chunks pipelined over three streams (H2D, compute, D2H).  A side
    # figure, never `value`.
    pcie = None
    if rank == 0 and world == 1 and args.pcie_chunks > 0 and B >= 2 * args.pcie_batch:
        pcie = pcie_inclusive(plan, a, b, c, args.pcie_batch, args.pcie_chunks, dev)

    # CPU baseline: the oracle (C, OpenMP over batch x towers) on a bounded sample
    cpu = None
    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import numpy as np
        import oracle as O

        Bs = 4
        tbs = O.Tables(n, qs, roots)
        ca = O.uniform_dcrt(Bs, T, n, qs, 1)
        cb = O.uniform_dcrt(Bs, T, n, qs, 2)
        O.ntt_mul_intt(ca, cb, tbs)  # warm
        runs, t0 = 0, time.perf_counter()
        while True:
            O.ntt_mul_intt(ca, cb, tbs)
            runs += 1
            el = time.perf_counter() - t0
            if el >= args.cpu_seconds:
                break
        cpu = {"value": runs * Bs * T * n / el, "unit": "coeffs/s", "cores": int(O.lib().oracle_num_threads()),
               "kind": "port",
               "sample": f"{runs} runs x {Bs} polys x {T} towers x N=2^{log_n} ({el:.1f} s), "
                         f"oracle/ofhe_oracle.c OpenMP over batch x towers, host {socket.gethostname()}"}

    if rank == 0:
        out = {
            "metric": METRIC,
            "value": value,
            "unit": "coeffs/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "weak" if args.shard == "batch" else "strong",
            "vs_baseline": None,
            "dtype": "u64",
            "data": "synthetic: uniform residues mod q_t (torch random_ on device), a coeff form, b eval form",
            "config": ({"workload": f"configs[2]: N=2^{log_n}, towers={T}, batch={B} per GPU, "
                                    "c = INTT(NTT(a) (.) b)",
                        "log_n": log_n, "towers": T, "batch_per_gpu": B, "global_batch": B * world,
                        "parallelism": f"batch-sharded x{world} (no data-path collective)"}
                       if args.shard == "batch" else
                       {"workload": f"configs[3]: N=2^{log_n}, towers={T_total} split over {world} GPUs, "
                                    f"batch={B}, c = INTT(NTT(a) (.) b)",
                        "log_n": log_n, "towers": T_total, "towers_rank0": T, "global_batch": B,
                        "parallelism": f"tower-sharded x{world} (no data-path collective)"}),
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "kernel": dominant,
                         "kernel_ms": kms, "alg_bytes_per_launch": ALG_BYTES_PER_COEFF * coeffs_rank,
                         "valu_issue": valu},
            "pipeline_hbm_frac": value / world * ALG_BYTES_PER_COEFF / (HBM_PEAK_GBS * 1e9),
            "kernels_ms": kernels,
            "cpu_baseline": cpu,
            "pcie_inclusive": pcie,
            "parity_spot_check": parity,
            "evalkey_broadcast": bcast,
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        torch.cuda.synchronize()
        if comm is not None:
            comm.close()
        dist.barrier()
        dist.destroy_process_group()


def pcie_inclusive(plan, a, b, c, bc, chunks, dev):
    """c = INTT(NTT(a) (.) b) with a, b in pinned host memory and c returned to
    it: chunk i's H2D, chunk i-1's pipeline and chunk i-2's D2H overlap on three
    streams; device slots alternate over the first 2*bc entries of a, b, c.
    Returns coefficients/s over `chunks` chunks of `bc` polynomials."""
    import torch

    T, n = a.shape[1], a.shape[2]
    ha, hb, hc = (torch.empty((bc, T, n), dtype=torch.int64, pin_memory=True) for _ in range(3))
    ha.copy_(a[:bc])
    hb.copy_(b[:bc])
    s_in, s_run, s_out = (torch.cuda.Stream(dev) for _ in range(3))
    ev = {k: [torch.cuda.Event() for _ in range(2)] for k in ("in", "run", "out")}
    for k in ev:
        for e in ev[k]:
            e.record(torch.cuda.current_stream(dev))

    def go():
        for i in range(chunks):
            sl = i % 2
            da, db, dc = a[sl * bc:(sl + 1) * bc], b[sl * bc:(sl + 1) * bc], c[sl * bc:(sl + 1) * bc]
            s_in.wait_event(ev["run"][sl])          # chunk i-2 no longer reads da, db
            with torch.cuda.stream(s_in):
                da.copy_(ha, non_blocking=True)
                db.copy_(hb, non_blocking=True)
            ev["in"][sl].record(s_in)
            s_run.wait_event(ev["in"][sl])
            s_run.wait_event(ev["out"][sl])         # chunk i-2's c has left the device
            plan.ntt_mul_intt(da.data_ptr(), db.data_ptr(), dc.data_ptr(), bc, s_run.cuda_stream)
            ev["run"][sl].record(s_run)
            s_out.wait_event(ev["run"][sl])
            with torch.cuda.stream(s_out):
                hc.copy_(dc, non_blocking=True)
            ev["out"][sl].record(s_out)
        torch.cuda.synchronize(dev)

    go()  # warm (first pinned transfers, plan tables)
    t0 = time.perf_counter()
    go()
    el = time.perf_counter() - t0
    coeffs = chunks * bc * T * n
    return {"value": coeffs / el, "unit": "coeffs/s", "chunk_batch": bc, "chunks": chunks,
            "pcie_bytes_per_coeff": 24, "pcie_gbs": coeffs * 24 / el / 1e9,
            "note": "a, b pinned host -> HBM, pipeline, c -> pinned host; 3 streams, double-buffered"}


def bench_keyswitch(args):
    """configs[4]: N = 2^17, 48 Q towers, dnum = 3, P = 16 towers; KeySwitchCore
    (ModUp -> key inner product -> 2x ModDown) on a batch of ciphertext
    polynomials per GPU, weak-scaled by batch.  Prints one JSON line."""
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    import ofhe_hip as H
    import shard

    log_n, sq, sp, dnum = 17, 48, 16, 3
    n = 1 << log_n
    allq, allr = moduli_chain(log_n, sq + sp)
    q, rq, p, rp = allq[:sq], allr[:sq], allq[sq:], allr[sq:]
    B = args.ks_batch
    ctx = H.Context(local)
    ks = H.KeySwitch(ctx, log_n, q, rq, p, rp, dnum)
    _, beta = ks.digits(sq)
    g = torch.Generator(device=dev)
    g.manual_seed(0x5EED + rank)

    def uniform(shape, moduli):
        x = torch.empty(shape, dtype=torch.int64, device=dev)
        for t, m in enumerate(moduli):
            x[..., t, :].random_(0, m, generator=g)
        return x

    c = uniform((B, sq, n), q)
    kb = torch.empty((dnum, sq + sp, n), dtype=torch.int64, device=dev)
    ka = torch.empty_like(kb)
    if rank == 0 or world == 1:
        kb.copy_(uniform((dnum, sq + sp, n), q + p))
        ka.copy_(uniform((dnum, sq + sp, n), q + p))
    key_bcast, comm = None, None
    if world > 1:  # the evaluation key comes from rank 0 over RCCL (configs[3]/[4])
        bfn, backend, comm = shard.key_broadcaster(ctx, rank, world)
        bfn(kb, 0)
        bfn(ka, 0)
        key_bcast = {"backend": backend, "verified": shard.same_on_all_ranks(kb) and shard.same_on_all_ranks(ka)}
    o0 = torch.empty((B, sq, n), dtype=torch.int64, device=dev)
    o1 = torch.empty_like(o0)
    digits = torch.empty((B, beta, sq + sp, n), dtype=torch.int64, device=dev)
    ct = torch.empty((2, B, sq + sp, n), dtype=torch.int64, device=dev)
    st = torch.cuda.current_stream(dev)
    sptr = st.cuda_stream

    def step():
        ks.core(sq, c.data_ptr(), kb.data_ptr(), ka.data_ptr(), o0.data_ptr(), o1.data_ptr(), 0, B, sptr)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        elapsed = shard.max_over_ranks(elapsed, device=dev)
    # stage split with events on the launch stream
    stages = {}
    reps = max(2, min(args.steps, 5))
    calls = {
        "mod_up(precompute)": lambda: ks.precompute(sq, c.data_ptr(), digits.data_ptr(), B, sptr),
        "inner_product": lambda: ks.fast_core_ext(sq, digits.data_ptr(), kb.data_ptr(), ka.data_ptr(),
                                                  ct[0].data_ptr(), ct[1].data_ptr(), B, sptr),
        "mod_down(x2)": lambda: (ks.mod_down(sq, ct[0].data_ptr(), o0.data_ptr(), 0, B, sptr),
                                 ks.mod_down(sq, ct[1].data_ptr(), o1.data_ptr(), 0, B, sptr)),
    }
    for name, fn in calls.items():
        fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(reps):
            fn()
        e1.record(st)
        e1.synchronize()
        stages[name] = e0.elapsed_time(e1) / reps
    # minimum HBM words per ciphertext polynomial and tower-coefficient: read c
    # (Q), write + read the digits (2 beta (Q+P)), write ct0/ct1 (2 (Q+P)),
    # ModDown reads them (2 (Q+P)) and writes out0/out1 (2 Q); keys are shared
    # by the batch and not counted
    qp = sq + sp
    alg_words = sq + 2 * beta * qp + 4 * qp + 2 * sq
    value = B * world * args.steps / elapsed
    if rank == 0:
        out = {
            "metric": "HYBRID key switches/sec (KeySwitchCore), N=2^17, 48+16 towers, dnum=3",
            "value": value, "unit": "keyswitch/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "u64", "data": "synthetic: uniform ciphertext and key residues",
            "config": {"workload": "configs[4]: N=2^17, Q=48, P=16, dnum=3, KeySwitchCore",
                       "batch_per_gpu": B, "global_batch": B * world,
                       "parallelism": f"ciphertext-batch-sharded x{world}, key broadcast over RCCL"},
            "stages_ms": stages,
            "alg_hbm_gbs": alg_words * 8 * n * B / (elapsed / args.steps) / 1e9,
            "evalkey_broadcast": key_bcast,
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        torch.cuda.synchronize()
        if comm is not None:
            comm.close()
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
