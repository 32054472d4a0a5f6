"""Summarise tools/pmc_stall.sh per pipeline kernel (medians over dispatches).

Units: SQ_WAVE_CYCLES, SQ_ACTIVE_INST_*, SQ_WAIT_* count quad-cycles summed
over waves; SQ_INSTS_* count wave-instructions; GRBM_GUI_ACTIVE counts GPU
cycles per XCD (summed over the 8 XCDs).  Derived, per kernel:
  clock_ghz        GRBM_GUI_ACTIVE / 8 / kernel time
  valu_issue       SQ_INSTS_VALU / (1024 SIMDs x clock cycles of the kernel)
  valu_active      SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES (share of a wave's life issuing VALU)
  dual_issue       SQ_ACTIVE_INST_VALU2 x 4 / SIMD cycles (share of SIMD cycles issuing two VALU ops)
  wait_any, wait_inst    SQ_WAIT_ANY, SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES
  waves_per_simd   SQ_WAVE_CYCLES x 4 / SIMD cycles (average resident waves)
"""
import csv
import glob
import json
import os
import sys

d = sys.argv[1]
NAMES = {"k_block<2,": "k_block<fused>", "k_block<0,": "k_block<fwd>", "k_block<1,": "k_block<inv>", "k_tcols<false": "colpass<fwd>", "k_tcols<true": "colpass<inv>"}


def kname(n):
    return next((v for k, v in NAMES.items() if k in n), None)


def med(v):
    v = sorted(v)
    return v[len(v) // 2] if v else None


def load(p):
    acc, dur = {}, {}
    for f in glob.glob(os.path.join(d, p, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = kname(r.get("Kernel_Name", ""))
            if k:
                key = (r.get("Dispatch_Id") or r.get("Correlation_Id") or ""), r["Counter_Name"]
                acc.setdefault(k, {}).setdefault(key, 0.0)
                acc[k][key] += float(r["Counter_Value"])
    for f in glob.glob(os.path.join(d, p, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = kname(r.get("Kernel_Name", ""))
            if k:
                dur.setdefault(k, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
    out = {}
    for k, m in acc.items():
        by = {}
        for (_, c), v in m.items():
            by.setdefault(c, []).append(v)
        out[k] = {c: med(v) for c, v in by.items()}
    return out, {k: med(v) for k, v in dur.items()}


res = {}
for p in ("a", "b", "c"):
    cs, du = load(p)
    for k, m in cs.items():
        e = res.setdefault(k, {})
        t = du.get(k)
        clk = m.get("GRBM_GUI_ACTIVE", 0) / 8 / t if t else None
        for c, v in m.items():
            if c != "GRBM_GUI_ACTIVE":
                e[c] = v
        e.setdefault("kernel_ms", {})[p] = t * 1e3 if t else None
        e.setdefault("clock_ghz", {})[p] = clk / 1e9 if clk else None
for k, e in res.items():
    t = e["kernel_ms"].get("b") or e["kernel_ms"].get("a")
    clk = (e["clock_ghz"].get("b") or e["clock_ghz"].get("a")) * 1e9
    simd_cycles = 1024 * clk * t * 1e-3
    der = {}
    if "SQ_INSTS_VALU" in e:
        der["valu_issue_per_simd_cycle"] = e["SQ_INSTS_VALU"] / simd_cycles
    if "SQ_WAVE_CYCLES" in e:
        wc = e["SQ_WAVE_CYCLES"]
        ta, ca = e["kernel_ms"].get("a"), e["clock_ghz"].get("a")
        sc_a = 1024 * ca * 1e9 * ta * 1e-3 if ta and ca else simd_cycles
        der["waves_per_simd"] = wc * 4 / sc_a
        for c in ("SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY"):
            if c in e:
                der[c.lower() + "_per_wave_cycle"] = e[c] / wc
        if "SQ_ACTIVE_INST_VALU2" in e:
            der["dual_issue_share_of_simd_cycles"] = e["SQ_ACTIVE_INST_VALU2"] * 4 / sc_a
    if "SQ_INSTS_VALU_INT64" in e and "SQ_INSTS_VALU" in e:
        der["int64_share"] = e["SQ_INSTS_VALU_INT64"] / e["SQ_INSTS_VALU"]
        der["int32_share"] = e["SQ_INSTS_VALU_INT32"] / e["SQ_INSTS_VALU"]
    e["derived"] = der
json.dump(res, sys.stdout, indent=1)
print()
