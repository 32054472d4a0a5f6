#!/bin/bash
# PMC passes for the roofline object of bench.py (profiles/pmc_current.json):
# HBM traffic (FETCH_SIZE and WRITE_SIZE, separate passes: MI355X_MICROARCH.md
# §HBM) and VALU issue (SQ_INSTS_VALU with GRBM_GUI_ACTIVE for the clock), each
# a kernel-trace-only rocprofv3 run of the headline configuration.  Usage:
#   tools/pmc_round.sh <tag>      -> gpurun_out/pmc_<tag>/ and gpurun_out/pmc_<tag>.json
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-current}"
OUT="$R/gpurun_out/pmc_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
pass() {  # name, counters...
  local name="$1"; shift
  timeout -s KILL ${PMC_TIMEOUT:-240} rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d "$OUT/$name" -o run \
      -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-extras --no-check ${PMC_ARGS} \
      > "$OUT/$name.stdout" 2> "$OUT/$name.err" || { echo "pmc pass $name failed rc=$?"; tail -5 "$OUT/$name.err"; exit 1; }
  echo "pmc pass $name done"
}
pass fetch FETCH_SIZE
pass write WRITE_SIZE
pass valu SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE
pass lds SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE
python3 "$R/tools/pmc_round_summarize.py" "$OUT" > "$R/gpurun_out/pmc_$TAG.json" && cat "$R/gpurun_out/pmc_$TAG.json"
