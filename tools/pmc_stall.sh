#!/bin/bash
# Where the pipeline kernels' cycles go: issue, dual issue, waits, VMEM / LDS
# FIFO stalls, 32- vs 64-bit integer instruction mix.  Each pass is its own
# kernel-trace-only rocprofv3 run of the headline configuration (<= 8 SQ
# counters per pass, MI355X_MICROARCH.md §HBM/rocprofv3).  Usage:
#   tools/pmc_stall.sh <tag>  -> gpurun_out/pmcs_<tag>/ and gpurun_out/pmcs_<tag>.json
# STALL_OP=fwd|inv profiles the standalone transforms instead (tools/run_pipeline.py,
# configs[2] shape, RUN_BATCH / RUN_REPS from the environment).
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-current}"
OUT="$R/gpurun_out/pmcs_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
if [ -n "$STALL_OP" ]; then
  export RUN_OP="$STALL_OP" RUN_BATCH="${RUN_BATCH:-1024}" RUN_REPS="${RUN_REPS:-3}"
  CMD=("$R/tools/run_pipeline.py")
else
  CMD=("$R/bench.py" --steps 2 --warmup 1 --no-extras --no-check ${PMC_ARGS})
fi
pass() {  # name, counters...
  local name="$1"; shift
  timeout -s KILL ${PMC_TIMEOUT:-240} rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d "$OUT/$name" -o run \
      -- python3 "${CMD[@]}" \
      > "$OUT/$name.stdout" 2> "$OUT/$name.err" || { echo "pmc pass $name failed rc=$?"; tail -5 "$OUT/$name.err"; exit 1; }
  echo "pmc pass $name done"
}
pass a SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE
pass b SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM GRBM_GUI_ACTIVE
pass c SQ_THREAD_CYCLES_VALU SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE
python3 "$R/tools/pmc_stall_summarize.py" "$OUT" > "$R/gpurun_out/pmcs_$TAG.json" && cat "$R/gpurun_out/pmcs_$TAG.json"
