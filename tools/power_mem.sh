#!/bin/bash
# Package power and sclk while tools/power_mem.py streams copies of a given size.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p "$R/gpurun_out"
OUT="$R/gpurun_out/power_mem.txt"
: > "$OUT"
for mib in ${SIZES:-4096 64 2}; do
  (timeout -k 5 60 python "$R/tools/power_mem.py" $mib 8 > "$R/gpurun_out/mem_$mib.txt" 2>&1) &
  BP=$!
  sleep 5
  S=$(timeout 10 rocm-smi --showpower --showclocks 2>/dev/null | grep -E "sclk|fclk|Package Power" | tr -s ' ' | tr '\n' ' ')
  wait $BP || { echo "size $mib failed"; cat "$R/gpurun_out/mem_$mib.txt"; exit 1; }
  echo "$(cat "$R/gpurun_out/mem_$mib.txt") | $S" >> "$OUT"
done
cat "$OUT"
