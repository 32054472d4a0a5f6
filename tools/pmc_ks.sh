#!/bin/bash
# PMC pass (kernel-trace only) over the key-switch bench (configs[4], serial
# streams): VALU instructions, busy cycles and waits per kernel, summarised
# per kernel name.  Output: gpurun_out/pmc_ks/ and its summary on stdout.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/pmc_ks"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
export BENCH_KS_SINGLE_STREAM=1
pass() {  # name, counters...
  local name="$1"; shift
  timeout -s KILL 240 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d "$OUT/$name" -o run \
      -- python3 "$R/bench.py" --workload keyswitch --steps 3 --warmup 1 --no-check \
      > "$OUT/$name.stdout" 2> "$OUT/$name.err" || { echo "pass $name failed"; tail -5 "$OUT/$name.err"; exit 1; }
}
pass p1 SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE
pass p2 FETCH_SIZE
pass p3 WRITE_SIZE
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
n = collections.Counter()
dur = collections.defaultdict(float)
for f in glob.glob(out + "/p1/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        dur[r["Kernel_Name"][:48]] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
for f in glob.glob(out + "/p[123]/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"][:48]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, d in sorted(agg.items(), key=lambda kv: -dur.get(kv[0], 0)):
    t = dur.get(k, 0)
    cyc = d.get("GRBM_GUI_ACTIVE", 0) / 8
    clk = cyc / t / 1e9 if t else 0
    issue = d.get("SQ_INSTS_VALU", 0) / (1024 * cyc) if cyc else 0
    print(f"{k:48s} time {t*1e3:8.2f} ms  clock {clk:4.2f} GHz  VALU issue/SIMD-cycle {issue:5.3f}  "
          f"waves {d.get('SQ_WAVES', 0):9.0f}  wait/wave-cycle {d.get('SQ_WAIT_INST_ANY', 0) / max(1, d.get('SQ_WAVE_CYCLES', 1)):5.2f}  "
          f"HBM read {2 * d.get('FETCH_SIZE', 0) * 1024 / 1e9:7.2f} GB  write {d.get('WRITE_SIZE', 0) * 1024 / 1e9:7.2f} GB")
PY
