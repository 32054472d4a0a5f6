"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE runs of bench.py into
per-kernel HBM bytes per launch (profiles/pmc_traffic.json format).
gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE reads 1/2 of the bytes
of a wide coalesced streaming read, so the read side is doubled; WRITE_SIZE is
exact for 16-B streaming stores.  Units: counters are KiB."""
import csv
import glob
import json
import os
import sys

d = sys.argv[1]
NAMES = {"k_block<2,": "k_block<fused>", "k_tcols<false": "colpass<fwd>", "k_tcols<true": "colpass<inv>",
         "k_cols<4, false": "colpass<fwd>", "k_cols<4, true": "colpass<inv>"}
out = {"source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes) on bench.py --steps 2",
       "correction": "hbm_bytes = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (gfx950 FETCH_SIZE halving)",
       "kernels": {}}
vals = {}
for cnt in ("FETCH_SIZE", "WRITE_SIZE"):
    files = glob.glob(os.path.join(d, cnt, "**", "*counter_collection.csv"), recursive=True)
    for f in files:
        for r in csv.DictReader(open(f)):
            name = r.get("Kernel_Name", "")
            key = next((v for k, v in NAMES.items() if k in name), None)
            if key is None or r.get("Counter_Name") != cnt:
                continue
            vals.setdefault(key, {}).setdefault(cnt, []).append(float(r["Counter_Value"]))
cfg = {}
try:
    b = json.load(open(os.path.join(d, "FETCH_SIZE.stdout")))
    cfg = b["config"]
except Exception:
    pass
for k, v in vals.items():
    fs = v.get("FETCH_SIZE", [])
    ws = v.get("WRITE_SIZE", [])
    if not fs or not ws:
        continue
    f = sorted(fs)[len(fs) // 2] * 1024
    w = sorted(ws)[len(ws) // 2] * 1024
    out["kernels"][k] = {"fetch_bytes_raw": f, "write_bytes": w, "hbm_bytes_per_launch": 2 * f + w,
                         "launches": len(fs), "log_n": cfg.get("log_n"), "towers": cfg.get("towers"),
                         "batch": cfg.get("batch_per_gpu")}
print(json.dumps(out, indent=1))
