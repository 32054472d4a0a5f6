"""CPU checks of bench.py's launch contract and roofline bookkeeping (no GPU):
--gpus N starts N ranks itself (torch.distributed.run, gloo for the check),
WORLD_SIZE disagreeing with --gpus is an error, and the roofline object uses
PMC counters only when they measured this build and configuration."""
import json
import os
import subprocess
import sys

from conftest import ROOT

BENCH = os.path.join(ROOT, "bench.py")


def _env():
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    return env


def test_gpus_flag_starts_that_many_ranks():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--launch-check"], capture_output=True, text=True,
                       timeout=240, env=_env())
    assert r.returncode == 0, r.stderr[-2000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(line) == 1, r.stdout
    out = json.loads(line[0])
    assert out["n_gpus"] == 2 and sorted(out["ranks"]) == [0, 1] and sorted(out["local_ranks"]) == [0, 1]
    assert len(set(out["pids"])) == 2


def test_world_size_mismatch_is_an_error():
    env = dict(_env(), WORLD_SIZE="3", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2"], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 2
    assert "must agree" in r.stderr


def test_roofline_uses_only_matching_counters(tmp_path, monkeypatch):
    import bench

    kms = {"colpass<fwd>": 3.2, "k_block<fused>": 6.8, "colpass<inv>": 3.4}
    coeffs = 1024 * 16 * 65536
    monkeypatch.setattr(bench, "PMC_FILE", str(tmp_path / "none.json"))
    r = bench.make_roofline(13.5, kms, coeffs, 16, 16, 1024, ms_per_step=13.6)
    assert r["bound"] is None and r["valu"] is None and r["traffic"] is None
    # top level (schema 3): the metric op, 24 algorithmic B per coefficient over
    # the timed region's ms per step -- the figure the north star's 0.40 is on
    assert r["schema"] == 3
    assert abs(r["frac"] - 24 * coeffs / 13.6e-3 / 8e12) < 1e-12
    assert r["pipeline_frac"] == r["frac"] and abs(r["achieved"] / 8000 - r["frac"]) < 1e-12
    # the dominant kernel beside it: its algorithmic bytes over its launch time
    assert r["dominant_kernel"] == "k_block<fused>"
    assert abs(r["dominant_kernel_frac"] - 24 * coeffs / 6.8e-3 / 8e12) < 1e-12
    # without ms_per_step the op's event time stands in
    assert abs(bench.make_roofline(13.5, kms, coeffs, 16, 16, 1024)["frac"] - 24 * coeffs / 13.5e-3 / 8e12) < 1e-12
    pm = {"build_id": bench.build_id(), "config": {"log_n": 16, "towers": 16, "batch": 1024},
          "kernels": {k: {"hbm_bytes_per_launch": bench.KERNEL_BYTES[k] * coeffs, "valu_insts_per_coeff": ipc,
                          "clock_ghz": 1.6} for k, ipc in zip(kms, (86, 181, 98))}}
    f = tmp_path / "pmc.json"
    f.write_text(json.dumps(pm))
    monkeypatch.setattr(bench, "PMC_FILE", str(f))
    r = bench.make_roofline(13.5, kms, coeffs, 16, 16, 1024, ms_per_step=13.5)
    assert r["counters"] == "matched" and r["bound"] == "valu"
    assert r["dominant_kernel_traffic"] == 24 * coeffs
    assert r["traffic"] == sum(bench.KERNEL_BYTES[k] * coeffs for k in kms)
    want = (86 + 181 + 98) * coeffs / 64 / (1024 * 1.6e9 * 0.25) * 1e3
    assert abs(r["valu"]["valu_bound_ms"] - want) < 1e-9 and abs(r["valu"]["frac"] - want / 13.5) < 1e-12
    assert abs(r["kernels"]["k_block<fused>"]["valu"]["valu_bound_ms"] -
               181 * coeffs / 64 / (1024 * 1.6e9 * 0.25) * 1e3) < 1e-9
    pm["build_id"] = "stale"
    f.write_text(json.dumps(pm))
    r = bench.make_roofline(13.5, kms, coeffs, 16, 16, 1024)
    assert r["valu"] is None and "stale" in r["counters"]
    pm["build_id"] = bench.build_id()
    pm["config"]["batch"] = 256
    f.write_text(json.dumps(pm))
    assert bench.make_roofline(13.5, kms, coeffs, 16, 16, 1024)["valu"] is None


def test_require_capi_comm_fires_on_fallback():
    """--require-capi-comm: the ranks print their JSON line, then exit non-zero
    when the evaluation key did not travel through ofhe_hip_bcast_evalkey (on
    a CPU box the C-ABI communicator cannot come up, so the ranks fall back to
    gloo together).  Without the flag the same run succeeds."""
    for flag, ok in (([], True), (["--require-capi-comm"], False)):
        r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--launch-check"] + flag, capture_output=True,
                           text=True, timeout=240, env=_env())
        line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
        assert len(line) == 1, (r.stdout, r.stderr[-2000:])
        out = json.loads(line[0])
        st = out["evalkey_broadcast_capi"]
        assert st["capi"] is False and st["reasons"] and "torch.distributed gloo" in st["reasons"][0]
        assert out["evalkey_broadcast"]["verified"] is True
        assert (r.returncode == 0) == ok, (flag, r.returncode, r.stderr[-2000:])


def test_launch_check_reports_every_rank():
    """Each rank's own communicator outcome reaches the line: on a CPU box no
    rank has a device context, so both appear under comm_failed with the
    error each one raised."""
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--launch-check"], capture_output=True, text=True,
                       timeout=240, env=_env())
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    ranks = out["evalkey_broadcast"]["ranks"]
    assert sorted(x["rank"] for x in ranks) == [0, 1]
    assert all(not x["comm"] and "no device context" in x["error"] for x in ranks)
    st = out["evalkey_broadcast_capi"]
    assert st["per_rank"]["launch_check"] == {"comm_up": [], "comm_failed": [0, 1]}
    assert any("rank 1: no device context" in why for why in st["reasons"])


def test_capi_status_bookkeeping():
    import bench

    # per-rank outcomes: rank 3 alone failed -> capi False, rank 3 named
    ranks = [{"rank": i, "comm": i != 3, "error": None if i != 3 else "ncclCommInitRank: unhandled"} for i in range(8)]
    st = bench.capi_status({"headline": {"backend": "torch.distributed nccl (C-ABI comm: peer)", "capi": False,
                                         "ranks": ranks}}, 8)
    assert st["capi"] is False
    assert st["per_rank"]["headline"] == {"comm_up": [0, 1, 2, 4, 5, 6, 7], "comm_failed": [3]}
    assert st["reasons"][-1] == "headline: rank 3: ncclCommInitRank: unhandled"
    up = [{"rank": i, "comm": True, "error": None} for i in range(8)]
    st = bench.capi_status({"headline": {"backend": "ofhe_hip_bcast_evalkey (RCCL)", "capi": True, "ranks": up}}, 8)
    assert st["capi"] is True and st["reasons"] == [] and st["per_rank"]["headline"]["comm_up"] == list(range(8))

    assert bench.capi_status({"headline": None}, 1)["capi"] is None
    good = {"backend": "ofhe_hip_bcast_evalkey (RCCL)", "capi": True}
    bad = {"backend": "torch.distributed nccl (C-ABI comm: x)", "capi": False}
    assert bench.capi_status({"headline": good, "keyswitch": good}, 8)["capi"] is True
    st = bench.capi_status({"headline": good, "keyswitch": bad}, 8)
    assert st["capi"] is False and st["reasons"] == ["keyswitch: torch.distributed nccl (C-ABI comm: x)"]
    assert bench.capi_exit_code(st, True) == 3 and bench.capi_exit_code(st, False) == 0
    assert bench.capi_exit_code(bench.capi_status({"headline": good}, 2), True) == 0


def test_power_sample_parses_rocm_smi(monkeypatch):
    """bench.power_sample reads the current package power (not the cap, which
    rocm-smi prints first), the cap and sclk from rocm-smi's text output."""
    import subprocess
    import types

    import torch

    import bench

    txt = ("GPU[0]\t\t: sclk clock level: 1: (1946Mhz)\n"
           "GPU[0]\t\t: Max Graphics Package Power (W): 1400.0\n"
           "GPU[0]\t\t: Current Socket Graphics Package Power (W): 1391.0\n")
    monkeypatch.setattr(subprocess, "run", lambda *a, **k: types.SimpleNamespace(stdout=txt))
    monkeypatch.setattr(torch.cuda, "synchronize", lambda *a, **k: None)
    monkeypatch.setattr(torch.cuda, "Event", lambda *a, **k: types.SimpleNamespace(record=lambda *a: None,
                                                                                  query=lambda: False))
    monkeypatch.setattr(bench.time, "sleep", lambda s: None)
    calls = []
    r = bench.power_sample(lambda: calls.append(1), 10.0, 0, seconds=0.5)
    assert r["package_w"] == 1391.0 and r["cap_w"] == 1400.0 and r["sclk_mhz"] == 1946.0 and r["under_load"]
    assert len(calls) == r["steps_queued"] == 50


def test_configs3_line_at_eight_ranks():
    """bench.py --gpus 8 --shard towers --towers 32 --batch 512 (configs[3]):
    rank 0 owns 4 towers, the block names them, and the line's evaluation-key
    broadcast record carries every rank's communicator outcome (the record
    shape test_launch_check_reports_every_rank checks end to end)."""
    import bench

    args = bench.parse_args(["--gpus", "8", "--shard", "towers", "--towers", "32", "--batch", "512"])
    c = bench.headline_config(args.shard, 8, args.log_n, args.towers, args.batch)
    assert c["towers_rank0"] == 4 and c["towers"] == 32 and c["global_batch"] == 512
    assert c["workload"].startswith("configs[3]") and "tower-sharded x8" in c["parallelism"]
    c = bench.headline_config("batch", 8, 16, 16, 1024)
    assert c["global_batch"] == 8 * 1024 and c["batch_per_gpu"] == 1024


def test_eight_rank_launch_reports_every_rank():
    """The driver's 8-GPU launch shape rehearsed on the CPU (gloo): --gpus 8
    starts eight ranks, each joins the group, the key broadcaster agrees on
    one backend across all of them and the line names all eight ranks'
    communicator outcomes."""
    r = subprocess.run([sys.executable, BENCH, "--gpus", "8", "--launch-check"], capture_output=True, text=True,
                       timeout=600, env=_env())
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    assert out["n_gpus"] == 8 and sorted(out["ranks"]) == list(range(8)) and len(set(out["pids"])) == 8
    assert sorted(x["rank"] for x in out["evalkey_broadcast"]["ranks"]) == list(range(8))
    assert out["evalkey_broadcast"]["verified"] is True
    assert out["evalkey_broadcast_capi"]["per_rank"]["launch_check"]["comm_failed"] == list(range(8))


def test_keyswitch_roofline_counts():
    """configs[4]'s key-switch bound (bench.keyswitch_roofline): 320 transforms
    per key switch at Q = 48, P = 16, dnum = 3 (ModUp: 3 digits x (16 INTT +
    48 NTT); each ModDown: 16 INTT + 48 NTT) and the inner product's 3.09 GB at
    batch 8 (keyswitch-hybrid.cpp:330-482)."""
    import bench

    n = 1 << 17
    r = bench.keyswitch_roofline(48, 16, 3, n, 8, 3.35, {"inner_product": 0.53}, 1.44e11, 1.40e11)
    assert r["transforms_per_keyswitch"] == {"ntt": 240, "intt": 80, "total": 320}
    assert r["inner_product"]["alg_bytes"] == 8 * n * 64 * (8 * 3 + 2 * 3 + 2 * 8) == 3087007744
    want = 8 * n * (240 / 1.44e11 + 80 / 1.40e11) * 1e3 + 3087007744 / 8e12 * 1e3
    assert abs(r["bound_ms"] - want) < 1e-9 and abs(r["frac"] - want / 3.35) < 1e-12
    # a lower level: l = 40 towers -> digits of 16, 16, 8
    r = bench.keyswitch_roofline(40, 16, 3, n, 1, 1.0, {}, 1e11, 1e11)
    assert r["transforms_per_keyswitch"]["intt"] == 40 + 32
    assert r["transforms_per_keyswitch"]["ntt"] == (40 - 14 + 16) * 0 + sum(40 - c + 16 for c in (14, 14, 12)) + 80


def test_hook_gate_matches_the_committed_crossover():
    """Policy::measured() in host/ofhe_openfhe_hooks.hpp is, entry by entry,
    the larger of the two tables tests/cpp/hook_crossover.cpp printed on the
    MI355X boxes (profiles/r06_hook_crossover.txt, r06m_hook_crossover.txt;
    kNever above every size)."""
    import re

    from conftest import ROOT

    pat = re.compile(r"/\*\s*(\w+)\s*\*/\s*\{([^}]*)\}")

    def table(text):
        return {m.group(1): [255 if v.strip() == "kNever" else int(v) for v in m.group(2).split(",")]
                for m in pat.finditer(text)}

    runs = [table(open(os.path.join(ROOT, "profiles", f)).read().split("# Policy::measured()")[1])
            for f in ("r06_hook_crossover.txt", "r06m_hook_crossover.txt")]
    want = {op: [max(a, b) for a, b in zip(runs[0][op], runs[1][op])] for op in runs[0]}
    hdr = open(os.path.join(ROOT, "upmem--openfhe_amd", "host", "ofhe_openfhe_hooks.hpp")).read()
    shipped = table(hdr.split("static Policy measured()")[1].split("for (int o = 0;")[0])
    assert len(want) == 10 and shipped == want
