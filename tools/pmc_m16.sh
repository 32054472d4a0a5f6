#!/bin/bash
# Two PMC passes (kernel-trace only) over tools/run_pipeline.py with the
# four-round matrix-core block pass (OFHE_BLOCK_M16=1): VALU / wait counters, then MFMA /
# LDS / VMEM counters, for k_block_m16 and k_block (run with OFHE_BLOCK_M16=0 for the butterfly pass).  Output:
# gpurun_out/pmc_m16/
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/pmc_m16_${OFHE_BLOCK_M16:-1}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
export OFHE_BLOCK_M16=${OFHE_BLOCK_M16:-1} RUN_BATCH=${RUN_BATCH:-256} RUN_REPS=2
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY \
    SQ_WAIT_INST_ANY SQ_INSTS_LDS GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d "$OUT/p1" -o run \
    -- python3 "$R/tools/run_pipeline.py" > "$OUT/p1.stdout" 2> "$OUT/p1.err" || { echo "pass 1 failed"; tail -5 "$OUT/p1.err"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT \
    SQ_ACTIVE_INST_LDS SQ_INST_LEVEL_VMEM SQ_WAVES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d "$OUT/p2" -o run \
    -- python3 "$R/tools/run_pipeline.py" > "$OUT/p2.stdout" 2> "$OUT/p2.err" || { echo "pass 2 failed"; tail -5 "$OUT/p2.err"; exit 1; }
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(out + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        agg[r["Kernel_Name"][:40]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    print(k)
    for c, v in sorted(d.items()):
        print("  %-28s %.4g" % (c, sum(v) / len(v)))
PY
