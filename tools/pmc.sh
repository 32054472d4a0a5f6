#!/bin/bash
# HBM traffic of the pipeline kernels from PMC counters, one counter group per
# pass (MI355X_MICROARCH.md: FETCH_SIZE and WRITE_SIZE cannot share a pass),
# kernel-trace only (no sys/runtime trace with --pmc).  Output: gpurun_out/pmc/
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p "$R/gpurun_out/pmc"
cd /tmp && export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 ${PMC_TIMEOUT:-300} rocprofv3 --pmc $C --kernel-trace --output-format csv \
      -d "$R/gpurun_out/pmc/$C" -o run -- python3 "$R/bench.py" --steps 2 --warmup 1 --cpu-seconds 0 --no-check --pcie-chunks 0 \
      ${PMC_ARGS} > "$R/gpurun_out/pmc/$C.stdout" 2> "$R/gpurun_out/pmc/$C.err" || { echo "pmc $C failed rc=$?"; exit 1; }
  echo "pmc $C done"
done
python3 "$R/tools/pmc_summarize.py" "$R/gpurun_out/pmc" > "$R/gpurun_out/pmc/pmc_traffic.json" && cat "$R/gpurun_out/pmc/pmc_traffic.json"
