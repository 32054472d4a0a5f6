#!/bin/bash
# SQ counters (issue / wait breakdown) for the pipeline kernels; one pass per
# counter set, kernel-trace only.  Usage: tools/pmc_valu.sh [lib.so ...]
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p "$R/gpurun_out/pmcv"
cd /tmp && export TMPDIR=/tmp
libs="$@"; [ -z "$libs" ] && libs="$R/upmem--openfhe_amd/lib/libofhe_hip.so"
i=0
for L in $libs; do
  case "$L" in /*) ;; *) L="$R/$L";; esac
  i=$((i+1))
  for SET in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU GRBM_GUI_ACTIVE" "SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM SQ_WAVES GRBM_GUI_ACTIVE"; do
    tag=$(echo $SET | cut -c1-12 | tr ' ' _)
    RUN_LIB=$L timeout -k 10 200 rocprofv3 --pmc $SET --kernel-trace --output-format csv -d "$R/gpurun_out/pmcv/v$i/$tag" -o run -- python3 "$R/tools/run_pipeline.py" > /dev/null 2>"$R/gpurun_out/pmcv/v$i.$tag.err" || { echo "fail $L $SET"; exit 1; }
  done
  echo "v$i=$L"
done
python3 "$R/tools/pmc_valu_summarize.py" "$R/gpurun_out/pmcv"
