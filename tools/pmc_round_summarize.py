"""Summarise tools/pmc_round.sh into the file bench.py reads (profiles/pmc_current.json):
per pipeline kernel, HBM bytes per launch and VALU lane-instructions per
coefficient at the measured clock, tagged with the build id and configuration
they were measured on.

  hbm_bytes_per_launch = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024
      (counters in KiB; gfx950 FETCH_SIZE reports half the bytes of wide
      coalesced streaming reads, MI355X_MICROARCH.md §HBM)
  valu_insts_per_coeff = SQ_INSTS_VALU * 64 / coefficients per launch
      (SQ_INSTS_VALU counts wave64 instructions)
  clock_ghz            = GRBM_GUI_ACTIVE / 8 XCDs / kernel time
  valu_issue_per_simd_cycle = SQ_INSTS_VALU / (1024 SIMDs * clock * time)
"""
import csv
import glob
import json
import os
import sys

d = sys.argv[1]
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

NAMES = {"k_block<2,": "k_block<fused>", "k_tcols<false": "colpass<fwd>", "k_tcols<true": "colpass<inv>",
         "k_cols<4, false": "colpass<fwd>", "k_cols<4, true": "colpass<inv>"}


def kname(n):
    return next((v for k, v in NAMES.items() if k in n), None)


def med(v):
    v = sorted(v)
    return v[len(v) // 2] if v else None


def counters(pass_dir):
    acc, dur = {}, {}
    for f in glob.glob(os.path.join(pass_dir, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = kname(r.get("Kernel_Name", ""))
            if k:
                acc.setdefault(k, {}).setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    for f in glob.glob(os.path.join(pass_dir, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = kname(r.get("Kernel_Name", ""))
            if k:
                dur.setdefault(k, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
    return ({k: {c: med(v) for c, v in cs.items()} for k, cs in acc.items()}, {k: med(v) for k, v in dur.items()})


cfg = json.load(open(os.path.join(d, "fetch.stdout")))["config"]
log_n, towers, batch = cfg["log_n"], cfg["towers"], cfg["batch_per_gpu"]
coeffs = batch * towers << log_n
fetch, _ = counters(os.path.join(d, "fetch"))
write, _ = counters(os.path.join(d, "write"))
valu, vdur = counters(os.path.join(d, "valu"))
lds, ldur = counters(os.path.join(d, "lds"))
out = {"build_id": bench.build_id(), "config": {"log_n": log_n, "towers": towers, "batch": batch},
       "source": "tools/pmc_round.sh: rocprofv3 --pmc, one counter group per pass, kernel-trace only, "
                 "bench.py --steps 2 --warmup 1 --no-extras",
       "formulas": __doc__.split("\n\n")[1].strip(), "kernels": {}}
for k in sorted(set(fetch) | set(valu)):
    e = {}
    f, w = fetch.get(k, {}).get("FETCH_SIZE"), write.get(k, {}).get("WRITE_SIZE")
    if f is not None and w is not None:
        e.update(fetch_bytes_raw=f * 1024, write_bytes=w * 1024, hbm_bytes_per_launch=2 * f * 1024 + w * 1024,
                 alg_bytes_per_launch=bench.KERNEL_BYTES[k] * coeffs)
    v, t = valu.get(k, {}), vdur.get(k)
    if v.get("SQ_INSTS_VALU") and v.get("GRBM_GUI_ACTIVE") and t:
        clk = v["GRBM_GUI_ACTIVE"] / 8 / t
        e.update(valu_insts_per_coeff=v["SQ_INSTS_VALU"] * 64 / coeffs, clock_ghz=clk / 1e9, kernel_ms_counted=t * 1e3,
                 valu_issue_per_simd_cycle=v["SQ_INSTS_VALU"] / (bench.SIMDS * clk * t))
        if v.get("SQ_WAVE_CYCLES"):
            e["active_inst_valu_per_wave_cycle"] = v.get("SQ_ACTIVE_INST_VALU", 0) / v["SQ_WAVE_CYCLES"]
    li = lds.get(k, {})
    if li.get("SQ_ACTIVE_INST_LDS"):
        e.update(lds_bank_conflict_cycles=li.get("SQ_LDS_BANK_CONFLICT"), lds_active_cycles=li["SQ_ACTIVE_INST_LDS"],
                 lds_insts=li.get("SQ_INSTS_LDS"))
    out["kernels"][k] = e
print(json.dumps(out, indent=1))
