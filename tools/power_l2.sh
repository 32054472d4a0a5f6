#!/bin/bash
# Package power and sclk while tools/microbench/mempower_bin streams
# read-modify-write passes whose footprint lives in the per-XCD L2, the
# Infinity Cache or HBM (same kernel shape for all three).
#   CONFIGS="wg:KiB:passes ..." bash tools/power_l2.sh
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p "$R/gpurun_out"
OUT="$R/gpurun_out/power_l2_summary.txt"
: > "$OUT"
# 1024 wg x 32 KiB = 32 MiB total = 4 MiB per XCD (L2 edge); 512 x 32 = 2 MiB per XCD (L2);
# 1024 x 128 KiB = 128 MiB (Infinity Cache); 1024 x 4 MiB = 4 GiB (HBM)
for c in ${CONFIGS:-512:32:64 1024:32:64 1024:128:16 1024:4096:1}; do
  IFS=: read -r wg kib passes <<< "$c"
  (timeout -k 5 30 "$R/tools/microbench/mempower_bin" $wg $kib $passes 7 > "$R/gpurun_out/l2_$c.txt" 2>&1) &
  BP=$!
  sleep 3
  S=$(timeout 10 rocm-smi --showpower --showclocks 2>/dev/null | grep -E "sclk|fclk|Package Power" | tr -s ' ' | tr '\n' ' ')
  sleep 1
  S2=$(timeout 10 rocm-smi --showpower 2>/dev/null | grep -E "Package Power" | tr -s ' ' | tr '\n' ' ')
  wait $BP || { echo "$c failed"; cat "$R/gpurun_out/l2_$c.txt"; exit 1; }
  echo "$(cat "$R/gpurun_out/l2_$c.txt") | $S | $S2" >> "$OUT"
done
cat "$OUT"
