"""Summarise tools/pmc_valu.sh: per pipeline kernel, the SQ issue breakdown.
SQ_WAVE_CYCLES / SQ_ACTIVE_* / SQ_WAIT_* count quad-cycles summed over waves;
WAVE_CYCLES = ACTIVE_INST_ANY + WAIT_INST_ANY + WAIT_ANY (disjoint,
MI355X_MICROARCH.md).  Effective clock = GRBM_GUI_ACTIVE / 8 / kernel time."""
import collections
import csv
import glob
import os
import sys


def kind(nm):
    if "k_block" in nm:
        return "block"
    if "cols" in nm:
        return "cols_i" if "<true" in nm else "cols_f"
    return None


import json

d = sys.argv[1]
report = {"source": "rocprofv3 --pmc SQ_* GRBM_GUI_ACTIVE on tools/run_pipeline.py (N=2^16, 16 towers, batch 256)",
          "note": "valu_inst_per_simd_cycle: SQ_INSTS_VALU / (1024 SIMDs x clock x time); a 4-cycle "
                  "wave64 instruction stream saturates a SIMD at 0.25", "kernels": {}}
names = {"block": "k_block<fused>", "cols_f": "colpass<fwd>", "cols_i": "colpass<inv>"}
for vdir in sorted(glob.glob(os.path.join(d, "v*"))):
    if not os.path.isdir(vdir):
        continue
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(list)
    for f in glob.glob(os.path.join(vdir, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = kind(r["Kernel_Name"])
            if k:
                acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for f in glob.glob(os.path.join(vdir, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = kind(r["Kernel_Name"])
            if k:
                dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
    print("==", os.path.basename(vdir))
    for k, cs in sorted(acc.items()):
        med = {c: sorted(v)[len(v) // 2] for c, v in cs.items()}
        t = sorted(dur[k])[len(dur[k]) // 2] if dur[k] else 0
        print(f"  {k}: t={t * 1e3:.3f} ms " + " ".join(f"{c}={v:.4g}" for c, v in sorted(med.items())))
        wc = med.get("SQ_WAVE_CYCLES")
        if wc:
            parts = [f"{c[3:]}/wave={med[c] / wc:.3f}" for c in
                     ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY", "SQ_ACTIVE_INST_VALU") if c in med]
            print("     " + " ".join(parts))
        if "GRBM_GUI_ACTIVE" in med and t:
            clk = med["GRBM_GUI_ACTIVE"] / 8 / t
            line = f"     clock={clk / 1e9:.2f} GHz"
            ent = {"clock_ghz": round(clk / 1e9, 3), "kernel_ms": round(t * 1e3, 4)}
            if "SQ_INSTS_VALU" in med:
                # VALU wave-instructions per SIMD per cycle (1024 SIMDs)
                ipc = med["SQ_INSTS_VALU"] / (1024 * clk * t)
                line += f" valu_inst/SIMD/cycle={ipc:.3f}"
                ent["valu_inst_per_simd_cycle"] = round(ipc, 4)
            if wc:
                for c in ("SQ_ACTIVE_INST_VALU", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY"):
                    if c in med:
                        ent[c[3:].lower() + "_per_wave_cycle"] = round(med[c] / wc, 4)
            report["kernels"].setdefault(names[k], ent)
            print(line)
with open(os.path.join(d, "pmc_valu.json"), "w") as f:
    json.dump(report, f, indent=1)
