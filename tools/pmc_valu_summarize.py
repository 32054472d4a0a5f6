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


d = sys.argv[1]
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
            if "SQ_INSTS_VALU" in med:
                # VALU wave-instructions per SIMD per cycle (1024 SIMDs)
                line += f" valu_inst/SIMD/cycle={med['SQ_INSTS_VALU'] / (1024 * clk * t):.3f}"
            print(line)
