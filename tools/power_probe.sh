#!/bin/bash
# Package power and sclk while one pipeline stage (or variant) runs back to
# back: tools/power_stage.py in the background, rocm-smi sampled every ~0.5 s.
#   tools/power_probe.sh <tag> <stage> <seconds> [ENV=VAL ...]
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=$1; shift
mkdir -p "$R/gpurun_out"
OUT="$R/gpurun_out/power_$TAG.txt"
: > "$OUT"
(timeout -k 10 120 python "$R/tools/power_stage.py" "$@" >> "$OUT" 2> "$R/gpurun_out/power_$TAG.err") &
BP=$!
sleep 3
for i in $(seq 1 30); do
  kill -0 $BP 2>/dev/null || break
  timeout 10 rocm-smi --showpower --showclocks 2>/dev/null | grep -E "sclk|Package Power" | tr -s ' ' | tr '\n' ' ' >> "$OUT"
  echo >> "$OUT"
  sleep 0.3
done
wait $BP; rc=$?
echo "rc=$rc" >> "$OUT"
python3 - "$OUT" <<'PY'
import re, sys
t = open(sys.argv[1]).read()
w = [float(x) for x in re.findall(r"Package Power \(W\): ([0-9.]+)", t)]
s = [float(x) for x in re.findall(r"sclk clock level: \d+: \((\d+)Mhz\)", t)]
w2, s2 = w[2:], s[2:]
line = [l for l in t.splitlines() if "ms per call" in l]
print(sys.argv[1].split("/")[-1], line[0] if line else "no timing",
      "| power W median %.0f max %.0f | sclk MHz median %.0f" % (sorted(w2)[len(w2) // 2] if w2 else 0, max(w2 or [0]),
                                                                sorted(s2)[len(s2) // 2] if s2 else 0))
PY
exit $rc
