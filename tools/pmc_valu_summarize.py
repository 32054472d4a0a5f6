import csv, glob, os, sys, collections
d = sys.argv[1]
for vdir in sorted(glob.glob(os.path.join(d, "v*"))):
    if not os.path.isdir(vdir):
        continue
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(vdir, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            nm = r["Kernel_Name"]
            key = "block" if "k_block" in nm else ("cols_f" if "false" in nm else ("cols_i" if "k_cols" in nm else None))
            if key:
                acc[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
    print("==", os.path.basename(vdir))
    for k, cs in acc.items():
        med = {c: sorted(v)[len(v) // 2] for c, v in cs.items()}
        wc = med.get("SQ_WAVE_CYCLES", 1)
        line = " ".join(f"{c}={v:.4g}" for c, v in sorted(med.items()))
        print(f"  {k}: {line}")
        if "SQ_ACTIVE_INST_VALU" in med:
            print(f"    valu_active/wave_cycles={med['SQ_ACTIVE_INST_VALU']/wc:.3f} wait_inst/wave={med.get('SQ_WAIT_INST_ANY',0)/wc:.3f} wait_any/wave={med.get('SQ_WAIT_ANY',0)/wc:.3f} active_any/wave={med.get('SQ_ACTIVE_INST_ANY',0)/wc:.3f}")
