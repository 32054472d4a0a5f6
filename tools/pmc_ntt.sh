#!/bin/bash
# One PMC pass (kernel-trace only) of the standalone forward / inverse NTT at
# N = 2^16 and 2^17 (tools/run_pipeline.py): VALU instructions per coefficient
# and issue rate per kernel, to compare the block pass at NR = 2 and NR = 3.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/pmc_ntt"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for cfg in "16 fwd 128" "17 fwd 64" "16 inv 128" "17 inv 64"; do
  set -- $cfg
  d="$OUT/n$1_$2"
  RUN_LOGN=$1 RUN_OP=$2 RUN_BATCH=$3 RUN_REPS=2 timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES \
      SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE --kernel-trace \
      --output-format csv -d "$d" -o run -- python3 "$R/tools/run_pipeline.py" > "$d.stdout" 2> "$d.err" \
      || { echo "pass $cfg failed"; tail -5 "$d.err"; exit 1; }
  python3 - "$d" $1 $3 <<'PY'
import csv, glob, sys, collections
d, logn, B = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
coefs = B * 16 << logn
agg = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter(); dur = collections.defaultdict(float)
for f in glob.glob(d + "/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "ofhe" in r["Kernel_Name"]:
            dur[r["Kernel_Name"][:44]] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
            n[r["Kernel_Name"][:44]] += 1
for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "ofhe" in r["Kernel_Name"]:
            agg[r["Kernel_Name"][:44]][r["Counter_Name"]] += float(r["Counter_Value"])
for k, c in agg.items():
    cyc = c["GRBM_GUI_ACTIVE"] / 8
    print(f"N=2^{logn} {k:44s} ms/launch {dur[k] / n[k] * 1e3:7.3f} VALU/coef {c['SQ_INSTS_VALU'] * 64 / coefs / n[k]:6.1f} "
          f"issue {c['SQ_INSTS_VALU'] / (1024 * cyc):5.3f} clock {cyc / dur[k] / 1e9:4.2f} wait/wave-cycle {c['SQ_WAIT_INST_ANY'] / c['SQ_WAVE_CYCLES']:4.2f}")
PY
done
