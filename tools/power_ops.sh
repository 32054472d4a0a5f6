#!/bin/bash
# Package power and sclk per VALU instruction type (tools/microbench/oppower_bin,
# built in-tree): each op runs back to back for 6 s; rocm-smi sampled mid-run.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p "$R/gpurun_out"
OUT="$R/gpurun_out/power_ops.txt"
: > "$OUT"
for op in ${OPS:-add_u32 xor_b32 add_co_u32 cndmask_b32 mul_lo_u32 mul_hi_u32 mul_u32_u24 mad_u64_u32 lshl_add_u64 mov_b64 fma_f32 fma_f64}; do
  (timeout -k 5 30 "$R/tools/microbench/oppower_bin" $op 6 > "$R/gpurun_out/op_$op.txt" 2>&1) &
  BP=$!
  sleep 3
  S=$(timeout 10 rocm-smi --showpower --showclocks 2>/dev/null | grep -E "sclk|Package Power" | tr -s ' ' | tr '\n' ' ')
  sleep 1
  S2=$(timeout 10 rocm-smi --showpower 2>/dev/null | grep -E "Package Power" | tr -s ' ' | tr '\n' ' ')
  wait $BP || { echo "$op failed"; cat "$R/gpurun_out/op_$op.txt"; exit 1; }
  echo "$(cat "$R/gpurun_out/op_$op.txt") | $S | $S2" >> "$OUT"
done
cat "$OUT"
