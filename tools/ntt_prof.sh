#!/bin/bash
R="${GRAFT_REPO_ROOT}"
cd /tmp && export TMPDIR=/tmp
for op in fwd inv; do
  RUN_OP=$op RUN_BATCH=1024 RUN_REPS=5 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/ntt_$op" -o run -- python3 "$R/tools/run_pipeline.py" > "$R/gpurun_out/ntt_$op.out" 2>&1 || exit 1
  RUN_OP=$op RUN_BATCH=1024 RUN_REPS=3 timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE SQ_WAVE_CYCLES --kernel-trace --output-format csv -d "$R/gpurun_out/ntt_${op}_pmc" -o run -- python3 "$R/tools/run_pipeline.py" > "$R/gpurun_out/ntt_${op}_pmc.out" 2>&1 || exit 1
done
echo ok
